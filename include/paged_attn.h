/*
 * paged_attn.h — C ABI of libpaged-attention.so, MI355X (gfx950) build.
 *
 * Drop-in for the reference's public header `csrc/paged_attn.h` (installed to
 * include/ by CMakeLists.txt:78-81): the three reference entry points keep their
 * exact names, parameter order and types.  Everything else here is new.
 *
 * Conventions shared by every entry point (reference semantics):
 *   - all pointers are caller-owned DEVICE pointers on the current HIP device;
 *     tensors are contiguous: dense  [batch, seqlen, heads, head_size],
 *     varlen [total_tokens, heads, head_size], paged [num_blocks, page, heads_k, head_size];
 *   - head_size must be a multiple of 8 (callers pad, export.cpp:539-547) and <= 256;
 *   - `is_fp16 == false` means bf16;
 *   - causality is carried ONLY by the windows: causal <=> window_left < 0 && window_right == 0
 *     (paged_attn.cpp:116); the `is_causal` flags of the varlen/paged entries are ignored,
 *     exactly as in the reference;
 *   - work is enqueued asynchronously on `stream`; nothing synchronises;
 *   - errors never throw or exit: the call returns without launching and the reason is
 *     readable from fmha_last_error() on the calling thread (""/NULL-free on success).
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

/* ABI 2.1: the entries whose argument lists changed in 2.0 are exported under _v2 names; these
 * macros keep sources that call the plain names compiling unchanged, while a binary built
 * against the 1.0 header fails to link instead of calling them with a stale argument list
 * (the pattern of the CUDA driver API's cuMemAlloc -> cuMemAlloc_v2). */
#define fmha_varlen_fwd_ex fmha_varlen_fwd_ex_v2
#define fmha_page_kvcache_fwd_ex fmha_page_kvcache_fwd_ex_v2
#define fmha_bwd_workspace_size fmha_bwd_workspace_size_v2
#define fmha_varlen_bwd_workspace_size fmha_varlen_bwd_workspace_size_v2
#define fmha_varlen_bwd fmha_varlen_bwd_v2

#ifdef __cplusplus
#define FMHA_DEFAULT(x) = x
extern "C" {
#else
#define FMHA_DEFAULT(x)
#endif

/* Dense forward.  Replaces csrc/paged_attn.h:8-31 (impl paged_attn.cpp:310-383).
 * Writes o and, when softmax_lse_ptr != NULL, the fp32 log-sum-exp [batch, heads, seqlen_q]
 * (the reference leaves it unwritten; bwd needs it).  alibi_slopes_ptr: fp32 [heads] or
 * [batch, heads] (the latter when batch > 1, as paged_attn.cpp:375 assumes).  p_dropout in
 * [0, 1): P is dropped with Philox keep bits drawn from this thread's RNG state
 * (fmha_set_rng_state) and the kept values scaled by 1 / (1 - p_dropout), as the reference's
 * dropout forward (dropout_hip.h:14-109, whose C path never runs it); no KV
 * split with dropout.  return_softmax (needs p_dropout > 0, p_ptr and softmax_lse_ptr): p_ptr
 * receives the dropped-out softmax [batch, heads, round128(seqlen_q), round128(seqlen_k)] in q's
 * dtype, dropped entries with the sign bit set (the reference's S_dmask encoding; here P is
 * normalised).  num_splits <= 0 picks a split count; 1 forces the single-pass kernel. */
void fmha_fwd(void* q_ptr, void* k_ptr, void* v_ptr, void* o_ptr, void* alibi_slopes_ptr,
              const int32_t seqlen_q, const int32_t seqlen_k, const int32_t batch_size,
              const int32_t num_heads, const int32_t num_heads_k, const int32_t head_size,
              const float p_dropout, hipStream_t stream, hipDeviceProp_t* dprops,
              const float softmax_scale, void* p_ptr, void* softmax_lse_ptr,
              int window_size_left, int window_size_right, const float softcap,
              const bool return_softmax, bool is_fp16, int num_splits FMHA_DEFAULT(0));

/* Varlen (packed, ragged) forward.  Replaces csrc/paged_attn.h:33-53 (impl
 * paged_attn.cpp:385-440).  cu_seqlens_{q,k}: int32 [batch+1], cumulative. */
void fmha_varlen_fwd(void* q_ptrs, void* k_ptrs, void* v_ptrs, void* o_ptrs,
                     void* cu_seqlens_q_ptrs, void* cu_seqlens_k_ptrs,
                     const int32_t max_seqlen_q, const int32_t max_seqlen_k,
                     const int32_t batch_size, const int32_t num_heads,
                     const int32_t num_heads_k, const int32_t head_size, hipStream_t stream,
                     const float softmax_scale, const bool is_causal, const bool is_fp16,
                     int window_size_left FMHA_DEFAULT(-1), int window_size_right FMHA_DEFAULT(-1));

/* Paged-KV forward (decode / chunked prefill over a block table).  Replaces
 * csrc/paged_attn.h:55-84 (impl paged_attn.cpp:442-568).
 * kcache/vcache [num_blocks, page_block_size, heads_k, head_size]; block_table int32
 * [batch, max_cache_seq_k / page_block_size]; cache_seqlens_k int32 [batch] = per-sequence
 * lengths (non-cumulative).  k/v (append), cache_batch_idx and rotary are ignored exactly
 * as in the reference C path (paged_attn.cpp:513-525).  Split scratch comes from a cached
 * per-device pool (no per-call hipMalloc, no leak — cf. paged_attn.cpp:186-189,557-561). */
void fmha_page_kvcache_fwd(void* q_ptr, void* kcache_ptr, void* vcache_ptr, void* k_ptr,
                           void* v_ptr, void* o_ptr, void* block_table_ptr,
                           void* cache_seqlens_k_ptr, const int32_t max_cache_seq_k,
                           const int32_t seqlen_q, const int32_t seqlen_k,
                           const int32_t batch_size, const int32_t num_heads,
                           const int32_t num_heads_k, const int32_t head_size,
                           const int32_t page_block_size, hipStream_t stream,
                           const float softmax_scale, int window_size_left,
                           int window_size_right, const int32_t num_splits,
                           void* cache_batch_idx_ptr, void* rotary_cos_ptr, void* rotary_sin_ptr,
                           bool is_causal, bool is_rotary_interleaved, bool is_fp16);

/* ---------------------------------------------------------------- new entry points --- */

/* Thread-local description of the last failed call on this thread ("" if none). */
const char* fmha_last_error(void);
/* 0 if the last call on this thread succeeded, a nonzero code otherwise. */
int fmha_last_status(void);

/* KV split count the last forward call on this thread launched with (1 = single pass; decode
 * kernel: one split per wave; 0 if that call launched nothing).  Diagnostic, for tests and
 * tuning. */
int fmha_last_num_splits(void);

/* The forward kernel the last forward call on this thread launched, with its schedule, e.g.
 * "fmha_fwd4_kernel persistent=2 xcdq=0 grid=256x1x1 block=256" ("" if the call launched no
 * forward kernel).  persistent: 0 one workgroup per item, 1 boustrophedon, 2 XCD-grouped item
 * pairs, 3 dynamic queue (xcdq=1: one queue per XCD).  Diagnostic (ABI 2.3), for tests and the
 * bench line; the combine launch of a split forward is not named. */
const char* fmha_last_kernel(void);

/* Dropout RNG state of the calling thread: the following forward / backward calls with
 * p_dropout > 0 draw their keep bits from Philox4x32-7 keyed by (seed, offset) over the score
 * coordinates (batch x head, query position, key) - a forward and the backward of the same
 * scores with the same state drop the same entries (flash-attn's rng_state = {seed, offset}). */
void fmha_set_rng_state(uint64_t seed, uint64_t offset);

/* Graph-capturable dropout key (ABI 2.2): the next dropout call on this thread reads its key
 * on the device when it runs - seed = *seed_ptr, offset = *offset_ptr + offset_add (torch's
 * philox_cuda_state under stream capture: seed_.ptr, offset_.ptr, offset_intragraph_, which the
 * reference unpacks in its kernels, flash_api_hip.cpp:509) - and a forward writes the key it used
 * to rng_out[0..1] (device int64 x 2, may be NULL; the reference's params.rng_state).  The
 * backward of that forward: fmha_set_rng_state_device(rng_out, rng_out + 1, 0, NULL).
 * seed_ptr == NULL keeps the host key of fmha_set_rng_state (rng_out still receives it).
 * One-shot: consumed by the next entry that takes p_dropout, whatever its value or outcome
 * (fmha_set_rng_state clears it too). */
void fmha_set_rng_state_device(const int64_t* seed_ptr, const int64_t* offset_ptr,
                               uint64_t offset_add, int64_t* rng_out);

/* Library version / build identification, e.g. "xf-fmha-gfx950 2.2".  2.0 (round 3) changed
 * argument lists of existing symbols; 2.1 exports those under _v2 names (see INTEGRATION.md
 * "ABI history"). */
const char* fmha_version(void);

/* Process-wide schedule knobs; every setting computes the same results (the parity suite runs
 * under any of them).  Each knob is an atomic value read once per call, so setting one while
 * another thread launches is safe (that launch sees the old or the new value).  Returns 0, or
 * -1 for an unknown name / out-of-range value.  Knobs: fwd_waves (4 | 8 waves = 128 | 256
 * query rows per forward workgroup), fwd_prio (0/1), fwd_persistent (workgroups per CU, 0 =
 * one workgroup per item), fwd_slack (0..16), fwd_order (0/1), fwd_dyn (0..2), fwd_xcdq (0/1),
 * fwd_pipe (0..2), fwd_decode (0/1), dec_wg_per_cu (1..16), dec_hmaj (0..2), dec_mr (16/32),
 * fwd_w4 (D = 128 forward where eligible — dense, varlen, or a paged cache whose page size is a
 * power of two >= 8: 4 auto, the default = 3 where no row has a right window and the cache is
 * not paged, else 2; 3 the 8-wave ping-pong kernel on the 16x16x32 MFMA (not paged); 2 the
 * 8-wave ping-pong kernel on 32x32x16; 1 the 4-wave kernel (variants build); 0 neither), fp8_w4 (fp8 forward: 1 the 4-wave kernel, the default; 2 the
 * 8-wave ping-pong kernel; 0 the 8-wave compiler-scheduled one), comb_row (0/1), bwd_order (0/1),
 * bwd_desc (0/1), dec_fold (0/1: the decode split combine folded into the split launch). */
int fmha_set_option(const char* name, int value);
/* Current value of a knob, or -1 (with fmha_last_error set) for an unknown name. */
int fmha_get_option(const char* name);

/* fp8 forward (extension; north_star "the two back-to-back GEMMs on ... fp8 MFMA"): q, k, v in
 * OCP fp8 e4m3fn ([batch, seqlen, heads, 128] contiguous bytes, as fmha_fwd's layout) with
 * per-tensor fp32 dequant scales (value = stored x scale, FA3's descale_q/k/v); both GEMMs on
 * the gfx950 block-scaled fp8 MFMA (2x the bf16 rate), P rounded to e4m3 for the PV product.
 * o: bf16 (out_fp16 = false) or fp16 [batch, seqlen_q, heads, 128]; softmax_lse fp32
 * [batch, heads, seqlen_q] or NULL.  Causality / windows as fmha_fwd (causal <=> wl < 0 &&
 * wr == 0).  head_size must be 128; no ALiBi / softcap / dropout. */
/* fmha_fwd with explicit ELEMENT strides for q, k, v, o (batch, row, head; the last dimension
 * is contiguous): head- or batch-sliced views run without a copy (the reference's C ABI assumes
 * contiguous tensors, csrc/paged_attn.cpp:46-60).  strides[12] = {q_batch, q_row, q_head,
 * k_batch, k_row, k_head, v_batch, v_row, v_head, o_batch, o_row, o_head}.  softmax_lse is
 * [batch, num_heads, seqlen_q] contiguous (or NULL).  head_size must be a multiple of 8.
 * p_dropout / s_dmask: dropout and return_softmax as fmha_fwd (s_dmask = its p_ptr, or NULL). */
void fmha_fwd_strided(void* q, void* k, void* v, void* o, void* alibi_slopes, void* softmax_lse,
                      int32_t seqlen_q, int32_t seqlen_k, int32_t batch_size, int32_t num_heads,
                      int32_t num_heads_k, int32_t head_size, const int64_t* strides,
                      float softmax_scale, int window_size_left, int window_size_right,
                      float softcap, bool is_fp16, int num_splits, hipStream_t stream,
                      float p_dropout, void* s_dmask);

void fmha_fwd_fp8(void* q, void* k, void* v, void* o, void* softmax_lse, float q_scale,
                  float k_scale, float v_scale, int32_t seqlen_q, int32_t seqlen_k,
                  int32_t batch_size, int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                  float softmax_scale, int window_size_left, int window_size_right, bool out_fp16,
                  hipStream_t stream);

/* Varlen forward with the fields the reference's varlen C entry drops (paged_attn.cpp:423-433):
 * LSE out (fp32 [num_heads, total_q], unpadded as export.cpp:827; total_q = cu_seqlens_q[batch]
 * must be passed by the caller, it is only used to address the LSE), ALiBi, softcap,
 * seqused_k (int32 [batch], optional), and an optional paged K/V (block_table != NULL: k/v are
 * [num_blocks, page, heads_k, head_size], block_table [batch, block_table_stride]).
 * p_dropout / s_dmask: as fmha_fwd (non-paged only; s_dmask [batch, heads,
 * round128(max_seqlen_q), round128(max_seqlen_k)], each sequence's rows from 0). */
void fmha_varlen_fwd_ex_v2(void* q, void* k, void* v, void* o, void* softmax_lse,
                        void* cu_seqlens_q, void* cu_seqlens_k, void* seqused_k,
                        void* block_table, int32_t block_table_stride, int32_t page_block_size,
                        void* alibi_slopes, int32_t alibi_batch_stride,
                        int32_t max_seqlen_q, int32_t max_seqlen_k, int32_t total_q,
                        int32_t batch_size, int32_t num_heads, int32_t num_heads_k,
                        int32_t head_size, float softmax_scale, int window_size_left,
                        int window_size_right, float softcap, bool is_fp16, hipStream_t stream,
                        float p_dropout, void* s_dmask);

/* Paged-KV forward that also returns LSE (fp32 [batch, num_heads, seqlen_q]) and takes ALiBi
 * and an fp8 (OCP e4m3fn) K/V cache with per-tensor dequant scales.
 * kv_dtype: 0 = same as q (fp16/bf16), 1 = fp8 e4m3fn (k_scale/v_scale multiply the stored
 * values).  num_splits <= 0 picks a split count.
 * cache_leftpad: optional int32 [batch_size] (flash-attn's leftpad_k, block_info.h; commented
 * out in export.cpp:1627-1634): batch b attends over cache rows [cache_leftpad[b],
 * cache_seqlens[b]), key positions counted from cache_leftpad[b].  Only for one page per
 * sequence (max_seqlen_k <= page_block_size), as the reference: no paged KV with leftpad. */
void fmha_page_kvcache_fwd_ex_v2(void* q, void* kcache, void* vcache, void* o, void* softmax_lse,
                              void* block_table, int32_t block_table_stride, void* cache_seqlens,
                              int32_t seqlen_q, int32_t max_seqlen_k, int32_t batch_size,
                              int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                              int32_t page_block_size, float softmax_scale,
                              int window_size_left, int window_size_right, float softcap,
                              void* alibi_slopes, int32_t alibi_batch_stride, int32_t num_splits,
                              int32_t kv_dtype, float k_scale, float v_scale,
                              void* cache_leftpad, bool is_fp16, hipStream_t stream);

/* KV-cache append with optional rotary embedding: the write step of mha_fwd_kvcache with new
 * k/v (export.cpp:1585-1669, kernel flash_fwd_kernel_hip.h:817-934 / rotary_hip.h:21-152 - never
 * enabled by the reference's C path, csrc/paged_attn.cpp:513-525).  For each batch b and new
 * token j: pos = cache_seqlens[b] + j; kcache/vcache slot (block_table[b][pos / page],
 * pos % page) <- rotary(knew[b][j]) / vnew[b][j]; seqlens_out[b] = cache_seqlens[b] +
 * seqlen_new.  With rotary_dim > 0 also q_out = rotary(q) at position cache_seqlens[b] + s
 * (q_rotary_per_token, the causal/local case) or cache_seqlens[b] (otherwise).  rotary_cos /
 * rotary_sin: [seqlen_ro, rotary_dim / 2] in q's dtype; interleaved = GPT-J pairs (2i, 2i+1),
 * else GPT-NeoX halves (i, i + rotary_dim/2).  knew/vnew contiguous [b, seqlen_new, hk, d];
 * caches contiguous [num_blocks, page, hk, d]; q/q_out contiguous [b, seqlen_q, h, d].
 * seqlens_out must be a different buffer from cache_seqlens (rejected otherwise: the kernel
 * reads the old lengths while writing the new ones).  New rows whose slot falls past the
 * block table's row (pos >= block_table_stride * page) are dropped.
 * Stream-ordered; run the attention (fmha_page_kvcache_fwd_ex with seqlens_out) after it. */
void fmha_kvcache_append(void* q, void* q_out, void* kcache, void* vcache, const void* knew,
                         const void* vnew, int32_t seqlen_new, const void* block_table,
                         int32_t block_table_stride, int32_t page_block_size,
                         const void* cache_seqlens, void* seqlens_out, const void* rotary_cos,
                         const void* rotary_sin, int32_t rotary_dim, bool is_rotary_interleaved,
                         bool q_rotary_per_token, int32_t batch_size, int32_t seqlen_q,
                         int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                         bool is_fp16, hipStream_t stream);

/* Dense backward: the C form of mha_bwd (export.cpp:948-1176, live twin flash_api_hip.cpp:
 * 815-1043), which the reference never built.  Inputs dout/q/k/v/out as the fwd layout,
 * softmax_lse fp32 [batch, heads, seqlen_q] from fmha_fwd; outputs dq [b,sq,h,d],
 * dk/dv [b,sk,hk,d] (GQA groups reduced in-kernel, no host sum_out), softmax_d fp32
 * [batch, heads, seqlen_q] (may be NULL: then pool scratch is used).  p_dropout: the forward's,
 * with the same fmha_set_rng_state (the keep bits are regenerated, not stored).
 * deterministic: S = min(ceil(CUs / (b * hk)), key blocks) fp32 dQ slices (the bound of
 * export.cpp:1086-1092), each owned by one workgroup that walks its key blocks in a fixed order
 * and adds by plain read-modify-write (D <= 128; D > 128: float atomics into the slice), then
 * summed in slice order: bitwise reproducible for a given S, instead of float atomics into one
 * accumulator.  S also stops at 1 + 8 GiB / (one slice's bytes).
 * workspace: optional caller scratch of fmha_bwd_workspace_size(..., deterministic) bytes;
 * NULL = pool.  A shorter workspace (at least one slice) is accepted and runs with as many
 * slices as it holds: still reproducible, but the dQ bits then depend on that slice count, so
 * pass the full size when results must match across callers.  One sequence's slab of any tensor must stay under 2 GiB - 256 bytes (32-bit
 * buffer offsets); larger inputs fail with an error, never a wrong result. */
void fmha_bwd(void* dout, void* q, void* k, void* v, void* out, void* softmax_lse,
              void* dq, void* dk, void* dv, void* alibi_slopes, void* softmax_d,
              int32_t seqlen_q, int32_t seqlen_k, int32_t batch_size, int32_t num_heads,
              int32_t num_heads_k, int32_t head_size, float p_dropout, float softmax_scale,
              int window_size_left, int window_size_right, float softcap, bool deterministic,
              bool is_fp16, hipStream_t stream, void* workspace, size_t workspace_bytes);

size_t fmha_bwd_workspace_size_v2(int32_t seqlen_q, int32_t seqlen_k, int32_t batch_size,
                               int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                               bool deterministic);

/* Varlen backward (mha_varlen_bwd semantics, flash_api_hip.cpp:1045-1298): packed q/k/v/out/
 * dout, cu_seqlens int32 [batch+1], softmax_lse fp32 [num_heads, total_q]; softmax_d fp32
 * [num_heads, total_q] receives rowsum(dO*O) (may be NULL: pool scratch).  deterministic and
 * workspace as fmha_bwd (fmha_varlen_bwd_workspace_size(..., deterministic) bytes); p_dropout as
 * fmha_bwd. */
void fmha_varlen_bwd_v2(void* dout, void* q, void* k, void* v, void* out, void* softmax_lse,
                     void* dq, void* dk, void* dv, void* cu_seqlens_q, void* cu_seqlens_k,
                     void* alibi_slopes, int32_t alibi_batch_stride, int32_t max_seqlen_q,
                     int32_t max_seqlen_k, int32_t total_q, int32_t total_k,
                     int32_t batch_size, int32_t num_heads, int32_t num_heads_k,
                     int32_t head_size, float softmax_scale, int window_size_left,
                     int window_size_right, float softcap, bool deterministic, bool is_fp16,
                     hipStream_t stream, void* workspace, size_t workspace_bytes,
                     void* softmax_d, float p_dropout);

size_t fmha_varlen_bwd_workspace_size_v2(int32_t total_q, int32_t max_seqlen_k, int32_t batch_size,
                                      int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                                      bool deterministic);

#ifdef __cplusplus
} /* extern "C" */
#endif
#undef FMHA_DEFAULT

// fmha_common.h — shared device/host definitions for the gfx950 attention kernels.
//
// Parameter blocks are our own POD structs (the reference packs `Flash_fwd_params`,
// csrc/flash_attn/src/flash_hip.h:50-172; we keep only what the MI355X kernels read).
// All strides are in ELEMENTS, like the reference (paged_attn.cpp:45-60).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <type_traits>

namespace xfa {

// Compile-time loop: f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>).
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}

// Per-device one-time host action (kernel attributes are set per device: a process may drive
// several GPUs).  `apply` runs once per (flag word, device) for devices 0..63 (always for
// others); the device's bit is set only after `apply` has returned, so a concurrent caller on
// the same device waits for it instead of launching before the attributes are in place.
template <typename F>
inline void once_per_device(std::atomic<unsigned long long>& done, int device, F&& apply) {
    if (device < 0 || device >= 64) { apply(); return; }
    const unsigned long long bit = 1ull << device;
    if (done.load(std::memory_order_acquire) & bit) return;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (done.load(std::memory_order_relaxed) & bit) return;
    apply();
    done.fetch_or(bit, std::memory_order_release);
}

// ------------------------------------------------------------------ vector types --
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// Raw buffer access (SRD in SGPRs, 32-bit per-lane byte offset, hardware range check):
// a load whose offset is past `bytes` returns zeros — used instead of `ok ? load : 0`
// selects, which hipcc lowers to a branch + vmcnt(0) drain per load.
constexpr int kOOB = 0x7FFFFF00;
// a wave-uniform pointer pinned to SGPRs (a buffer descriptor built from a base the compiler
// keeps in VGPRs turns its loads into waterfall loops)
__device__ __forceinline__ const char* uniform_ptr(const char* ptr) {
    const uint64_t a = (uint64_t)ptr;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return reinterpret_cast<const char*>(((uint64_t)hi << 32) | lo);
}
// (every descriptor here covers a wave-uniform range: base and size are pinned to SGPRs, a
// no-op where the compiler already has them there)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(uniform_ptr(reinterpret_cast<const char*>(base))),
                                             (short)0, __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}
__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, int voff) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
}
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
__device__ __forceinline__ u32x2 buf_load8(__amdgpu_buffer_rsrc_t r, int voff) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0);
}

constexpr int kBlockN = 64;   // keys per K/V tile (one LDS stage)
// forward LDS buffers per K/V tile pair and waves per SIMD, by head-dim bucket
constexpr int fwd_nbuf(int hd) { return hd > 128 ? 2 : 4; }
constexpr int fwd_waves_per_simd(int hd) { return hd > 128 ? 1 : 2; }
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ------------------------------------------------------------------ params -------
struct FwdParams {
    const void* q;
    const void* k;
    const void* v;
    void* o;
    float* lse;        // optional; index = b*lse_batch + h*lse_head + (q_offset + pos)
    float* oaccum;     // split scratch [splits][b][h][seqlen_q][HD] fp32
    float* lseaccum;   // split scratch [splits][b][h][seqlen_q] fp32

    int64_t q_batch, q_row, q_head;
    int64_t k_batch, k_row, k_head;   // paged: k_batch is the page stride
    int64_t v_batch, v_row, v_head;
    int64_t o_batch, o_row, o_head;
    int64_t lse_batch, lse_head;

    const int* cu_seqlens_q;   // varlen q (cumulative) or null
    const int* cu_seqlens_k;   // varlen k (cumulative) or null
    const int* seqused_k;      // per-batch key length (kvcache cache_seqlens / seqused_k) or null
    const int* leftpad_k;      // kvcache cache_leftpad [b] or null: keys [lp, seqused_k) of the
                               // cache are the sequence (key i = cache row lp + i)
    const int* block_table;    // paged K/V or null
    int bt_stride;
    int page_size;
    const float* alibi;        // fp32 slopes or null
    int alibi_bstride;

    int b, h, hk, group, d;
    int seqlen_q, seqlen_k;    // max lengths for varlen
    int wl, wr;                // normalised windows (<0 = unbounded)
    float scale_log2;          // multiplies the working score
    float softcap_pre;         // >0: w = tanh(s * softcap_pre)
    float alibi_mul;           // 1 / scale_softmax (bias in working units)
    int num_splits;
    int alibi_causal;          // the reference's is_causal with ALiBi: its LSE convention differs
    int kv_fp8;                // 1: K/V stored as fp8 e4m3fn
    float k_scale, v_scale;    // fp8 K/V dequant scales (stored value x scale)
    float q_scale;             // fp8 Q dequant scale (fp8 Q/K/V forward)
    int prio_hi;               // 1: waves NW/2.. run at s_setprio 1 (static, guide T5)
    int persistent;            // 1: persistent grid walking (row block, b*hk) items
    int n_mblocks;             // row blocks per (b, kv head) (persistent mode)
    int pipe;                  // 1: software-pipelined loop over the unmasked key tiles
    float max_slack;           // log2 units the running max may lag the true max before the
                               // O / l rescale (deferred rescale; 0 = rescale on every rise)
    int decode;                // 1: run fmha_decode_kernel (split-KV decode)
    int dec_mr;                // decode: 16 -> the 16x16x32 tile (query rows <= 16)
    int dec_hmaj;              // decode: the 4 waves of a workgroup are 4 kv heads of one split
    int* work_ctr;             // persistent == 3: self-resetting counters [-, finished, next x 8]
    int* dec_ctr;              // decode, combine folded in: per (batch, kv head) split arrival
                               // counters (zero between launches: the merging wave resets its own)
    int dec_bal;               // decode over ragged caches: split slots shared in proportion to
                               // the sequences' key tiles (fmha_decode_kernel.h dec_slot)
    int dec_slots, dec_cap;    // dec_bal: slots per kv-head group; max splits of one sequence
    int* dec_ns;               // dec_bal: [b] split count of each sequence (for the combine)
    int xcd_queues;            // persistent == 3: one item queue per XCD (else queue 0 only)
    // host-side launch choices (snapshotted from the options by the C ABI, per call)
    int waves;                 // 4 or 8 waves per workgroup (D <= 128)
    int num_cus;               // CUs of the current device
    int persist_per_cu;        // persistent workgroups per CU (0 = one workgroup per item)
    int order;                 // persistent item order (0 boustrophedon, 1 XCD-grouped pairs)
    int xcdq;                  // dynamic queue kind (1 per-XCD queues)
    int device;                // current device id (per-device one-time kernel attributes)
    int fwd4;                  // 1: the 4-wave D = 128 forward where eligible (fmha_fwd4_kernel.h)
    int comb_row;              // split combine: one workgroup per row when rows are few
    // dropout (flash_fwd_kernel_hip.h's Dropout, dropout_hip.h:14-109): keep a score iff its
    // Philox byte <= keep_thr (= floor(p_keep * 255), paged_attn.cpp:106-113); kept P scaled by
    // rp_keep = 1 / p_keep.  drop = 0: no dropout.
    int drop;
    uint32_t keep_thr;
    float rp_keep;
    uint64_t seed, offset;
    // graph-capturable key (fmha_set_rng_state_device): seed = *seed_ptr, offset = *offset_ptr
    // + offset, read on the device at run time; rng_out (forward): the key used, written back
    // for the backward as the reference's kernel writes params.rng_state
    const int64_t* seed_ptr;
    const int64_t* offset_ptr;
    int64_t* rng_out;
};

struct CombineParams {
    const float* oaccum;
    const float* lseaccum;
    void* o;
    float* lse;
    int64_t o_batch, o_row, o_head;
    int64_t lse_batch, lse_head;
    int b, h, seqlen_q, d, hd, num_splits;
    const int* dec_ns;   // per-batch split counts (balanced decode), or null: num_splits
};

struct BwdParams {
    const void* q; const void* k; const void* v; const void* o; const void* dout;
    const float* lse;
    void* dq; void* dk; void* dv;
    float* dq_accum;     // fp32 [b][h][seqlen_q_pad][HD] (varlen: [h][total_q_pad][HD])
    float* dsum;         // fp32 rowsum(dO*O), layout like lse

    int64_t q_batch, q_row, q_head;
    int64_t k_batch, k_row, k_head;
    int64_t v_batch, v_row, v_head;
    int64_t o_batch, o_row, o_head;
    int64_t do_batch, do_row, do_head;
    int64_t dq_batch, dq_row, dq_head;
    int64_t dk_batch, dk_row, dk_head;
    int64_t dv_batch, dv_row, dv_head;
    int64_t lse_batch, lse_head;   // lse / dsum index = b*lse_batch + h*lse_head + q_offset + pos
    int64_t acc_batch, acc_head, acc_row;  // dq_accum strides (floats)

    const int* cu_seqlens_q;
    const int* cu_seqlens_k;
    const float* alibi;
    int alibi_bstride;

    int b, h, hk, group, d;
    int seqlen_q, seqlen_k;
    int wl, wr;
    float scale;         // softmax scale (natural units)
    float scale_log2;
    float softcap_pre;
    float alibi_mul;
    int alibi_causal;    // causal ALiBi: the main kernel reads lse_fix (launch_lse_alibi)
    float* lse_fix;      // workspace [like lse]: the LSE back in the kernels' ALiBi convention
    int softcap_on;
    int dq_slices;       // deterministic: dQ partials per key block in dq_accum slices (0 = atomics)
    int64_t acc_slice;   // floats between dq_accum slices
    int device;          // current device id (per-device one-time kernel attributes)
    int order;           // 1: 1-D grid, the key blocks of one (batch, kv head) consecutive on one XCD
    int desc;            // 1: each key block sweeps its query tiles last to first
    // dropout (flash_fwd_kernel_hip.h's Dropout, dropout_hip.h:14-109): keep a score iff its
    // Philox byte <= keep_thr (= floor(p_keep * 255), paged_attn.cpp:106-113); kept P scaled by
    // rp_keep = 1 / p_keep.  drop = 0: no dropout.
    int drop;
    uint32_t keep_thr;
    float rp_keep;
    uint64_t seed, offset;
    // graph-capturable key (fmha_set_rng_state_device): seed = *seed_ptr, offset = *offset_ptr
    // + offset, read on the device at run time; rng_out (forward): the key used, written back
    // for the backward as the reference's kernel writes params.rng_state
    const int64_t* seed_ptr;
    const int64_t* offset_ptr;
    int64_t* rng_out;
};

// ------------------------------------------------------------------ dropout RNG --
// Philox4x32 with 7 rounds: the reference's philox() (philox.cuh:32-50, six rounds plus the
// final one, Weyl key bumps), here on a counter of the score's coordinates.
__device__ __forceinline__ u32x4 philox4x32_7(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1,
                                              uint32_t c2, uint32_t c3) {
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return u32x4{c0, c1, c2, c3};
}
// The random bytes of one 4 x 4 block of scores of (batch, head) bh = b * H + h: query positions
// 4 (pos >> 2) .. +3, keys 4 (key >> 2) .. +3.  Word i is query position 4 (pos >> 2) + i, its
// byte j key 4 (key >> 2) + j.  (A forward lane holds one query row and runs of 4 keys, a
// backward lane one key and runs of 4 query rows: both draw one block per run.)
// Keep a score iff its byte <= keep_thr.  Restated on the CPU by oracle/dropout_ref.py.
__device__ __forceinline__ u32x4 drop_block(const uint64_t seed, const uint64_t offset, const int bh,
                                            const int pos, const int key) {
    return philox4x32_7((uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(offset >> 32),
                        (uint32_t)key >> 2, (uint32_t)pos >> 2, (uint32_t)bh, (uint32_t)offset);
}
// The launch's Philox key: the host values, or (graph capture) the generator's device state, as
// the reference unpacks philox_cuda_state in its kernels (at::cuda::philox::unpack).
template <typename P>
__device__ __forceinline__ void drop_key(const P& p, uint64_t& seed, uint64_t& offset) {
    seed = p.seed;
    offset = p.offset;
    if (p.seed_ptr) {
        seed = (uint64_t)*p.seed_ptr;
        offset = (uint64_t)*p.offset_ptr + p.offset;
    }
}
__device__ __forceinline__ bool drop_keep(const uint32_t word, const int j, const uint32_t thr) {
    return ((word >> (8 * j)) & 0xFFu) <= thr;
}

// ------------------------------------------------------------------ dtype traits --
template <typename T> struct DT;
template <> struct DT<__bf16> {
    typedef bf16x8 v8;
    static __device__ __forceinline__ f32x16 mfma32(const v8& a, const v8& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
    typedef __attribute__((ext_vector_type(2))) __bf16 v2;
};
template <> struct DT<_Float16> {
    typedef f16x8 v8;
    static __device__ __forceinline__ f32x16 mfma32(const v8& a, const v8& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    typedef __attribute__((ext_vector_type(2))) _Float16 v2;
};

// Conflict-free 16-byte-chunk swizzle of a [rows][HD] 16-bit LDS tile (HD*2-byte rows),
// shared by the row reads (ds_read_b128, 32x32x16 A/B operand) and the transposed reads
// (ds_read_b64_tr_b16) — see DESIGN.md §LDS for the bank derivation.
template <int HD> __device__ __forceinline__ int swz(int row);
template <> __device__ __forceinline__ int swz<128>(int row) {
    return ((row & 3) << 2) | ((row >> 2) & 3);
}
template <> __device__ __forceinline__ int swz<64>(int row) {
    return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
}
// D = 256 rows are 512 B (also a whole number of bank rows): the D = 128 pattern on the low
// four chunk bits keeps the 32-row ds_read_b128 and the transposing reads conflict-free
template <> __device__ __forceinline__ int swz<256>(int row) {
    return ((row & 3) << 2) | ((row >> 2) & 3);
}
template <int HD> __device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * (HD * 2) + ((chunk ^ swz<HD>(row)) << 4);
}

// Forward K/V tile image: 8-row x 32-column subtiles of 512 B (cdna_hip_programming.md T10
// image (a)): byte offset of 16-byte chunk `chunk` of tile row `row`.  Conflict-free for the
// 32x32x16 row reads (ds_read_b128) and the transposed reads (ds_read_b64_tr_b16), like the
// plain-row XOR image, but a lane's reads then differ only by immediates except in one bit of
// the chunk (row reads) or of the row (transposed reads): two address registers per operand
// instead of NS (row reads) or 2*ND (transposed reads).  One LDS-DMA wave-instruction (1 KiB,
// lane l at +16 l) fills 8 rows x 8 chunks.
template <int HD> __device__ __forceinline__ int kv_off(int row, int chunk) {
    return (HD * 16) * (row >> 3) + 512 * (chunk >> 2) + 64 * (row & 7) +
           16 * ((chunk & 3) ^ ((row >> 2) & 3));
}

__device__ __forceinline__ float wave_max_halves(float x) {
    // lanes l and l^32 hold the same query row: exchange halves with v_permlane32_swap
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float wave_sum_halves(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// s_waitcnt immediate for gfx9: vmcnt(n) (6 bits, split [3:0] / [15:14]), expcnt and lgkmcnt
// left unconstrained.
__host__ __device__ constexpr int waitcnt_vm(int n) {
    return (n & 0xF) | ((n >> 4) << 14) | 0x0F70;
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// tanh without a libcall (a call would spill every live accumulator):
// tanh(x) = 1 - 2 / (exp(2x) + 1); saturates correctly at +-inf.
__device__ __forceinline__ float fast_tanh(float x) {
    const float e = __builtin_amdgcn_exp2f(x * (2.f * 1.4426950408889634f));
    return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

// Store one query row of the O^T accumulators (lane holds row lane&31, columns
// 32dt + 8g + 4hh .. +3 in registers 4g..4g+3 of acc[dt]) as 16-byte stores: pairs of column
// groups are exchanged between the lane halves with v_permlane32_swap so each lane writes 8
// contiguous columns (8 x 16 B per lane instead of 16 x 8 B; the tail is store-issue-bound,
// cdna_hip_programming.md T21).  Columns >= d (a multiple of 8) are not written.
template <typename T, int ND>
__device__ __forceinline__ void store_o_row16(T* orow, const f32x16 (&acc)[ND], float inv, int d, int hh) {
    typedef __attribute__((ext_vector_type(2))) T T2;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int gp = 0; gp < 4; gp += 2) {
            const T2 a0v = {(T)(acc[dt][4 * gp] * inv), (T)(acc[dt][4 * gp + 1] * inv)};
            const T2 a1v = {(T)(acc[dt][4 * gp + 2] * inv), (T)(acc[dt][4 * gp + 3] * inv)};
            const T2 b0v = {(T)(acc[dt][4 * gp + 4] * inv), (T)(acc[dt][4 * gp + 5] * inv)};
            const T2 b1v = {(T)(acc[dt][4 * gp + 6] * inv), (T)(acc[dt][4 * gp + 7] * inv)};
            const auto r0 = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a0v),
                                                             __builtin_bit_cast(unsigned, b0v), false, false);
            const auto r1 = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a1v),
                                                             __builtin_bit_cast(unsigned, b1v), false, false);
            const int col = 32 * dt + 8 * gp + 8 * hh;
            if (col < d) *reinterpret_cast<u32x4*>(orow + col) = u32x4{r0[0], r1[0], r0[1], r1[1]};
        }
}

// 8 OCP fp8 e4m3fn values (two dwords) -> 8 x T = T(f32(fp8) * scale), packed in 4 dwords.
template <typename T>
__device__ __forceinline__ u32x4 fp8x8_to(unsigned lo, unsigned hi, float scale) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    typedef __attribute__((ext_vector_type(2))) T T2;
    const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8(lo, false), b = __builtin_amdgcn_cvt_pk_f32_fp8(lo, true);
    const f2 c = __builtin_amdgcn_cvt_pk_f32_fp8(hi, false), d = __builtin_amdgcn_cvt_pk_f32_fp8(hi, true);
    const T2 ta = {(T)(a[0] * scale), (T)(a[1] * scale)}, tb = {(T)(b[0] * scale), (T)(b[1] * scale)};
    const T2 tc = {(T)(c[0] * scale), (T)(c[1] * scale)}, td = {(T)(d[0] * scale), (T)(d[1] * scale)};
    return u32x4{__builtin_bit_cast(unsigned, ta), __builtin_bit_cast(unsigned, tb),
                 __builtin_bit_cast(unsigned, tc), __builtin_bit_cast(unsigned, td)};
}

// fp8 e4m3fn (OCP) -> f32, exact.
__device__ __forceinline__ float fp8e4m3_to_f32(uint32_t b) {
    uint32_t s = (b & 0x80u) << 24;
    uint32_t e = (b >> 3) & 0xFu;
    uint32_t m = b & 0x7u;
    if (e == 0) {
        float f = (float)m * 0.001953125f;  // m * 2^-9
        return s ? -f : f;
    }
    if (e == 0xF && m == 0x7) return __uint_as_float(0x7FC00000u);
    return __uint_as_float(s | ((e + 120u) << 23) | (m << 20));
}

}  // namespace xfa

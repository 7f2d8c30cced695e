// fmha_launch.h — internal host-side launch interface (one object file per head dim x dtype).
// Replaces the reference's template fan-out run_mha_fwd_splitkv_dispatch / run_flash_splitkv_fwd
// (flash_fwd_launch_template_hip.h:106-189) and the bwd launch template
// (flash_bwd_launch_template_hip.h:76-136).
#pragma once

#include "fmha_common.h"

#include <atomic>

#ifndef XFA_VARIANTS
// 0: the product library.  1 (build.py --variants, lib/variants/): also the kernels no default
// path runs, kept for A/B and the bit-identity tests: the 4-wave D = 128 forward (fwd_w4 = 1) and
// the 8-wave ping-pong fp8 forward (fp8_w4 = 2)
#define XFA_VARIANTS 0
#endif

namespace xfa {

// Tuning knobs, settable through fmha_set_option() (schedule choices with equal results; the
// parity suite runs under any of them via XFA_TEST_OPTIONS).  Atomic: a launch on another
// thread reads each knob once, as a whole value.
struct Options {
    std::atomic<int> fwd_w4{4};          // D = 128 forward where eligible: 4 auto (3 where no row
                                         // has a right window, else 2); 3 the ping-pong on the
                                         // 16x16x32 MFMA (r6: non-causal C2 +1.5-2.8 %, causal
                                         // -1.3-3.4 % against 2, same box); 2 the 8-wave ping-pong
                                         // kernel (fmha_fwdpp_kernel.h; round 5, same box: C2 causal
                                         // +2-3 %, C4 +3 %, non-causal equal), 1 the 4-wave kernel
                                         // (fmha_fwd4_kernel.h), 0 neither (8-wave fmha_fwd_kernel)
    std::atomic<int> fp8_w4{1};          // 4-wave fp8 forward (fmha_fwd8w_kernel.h) where eligible
                                         // (C2 shape, same box: 1610 vs 1576 TFLOP/s causal, 1852 vs
                                         // 1799 non-causal)
    std::atomic<int> fwd_waves{8};       // waves per forward workgroup (4 or 8); 32 query rows per wave
    std::atomic<int> fwd_prio{0};        // static s_setprio 1 for the younger half of the workgroup
    std::atomic<int> fwd_persistent{1};  // persistent grid (workgroups per CU; 0 = one workgroup per item)
    std::atomic<int> fwd_slack{8};       // deferred rescale: running max may lag by this many log2 units
    std::atomic<int> fwd_order{1};       // persistent item order: 0 boustrophedon, 1 XCD-grouped pairs
    std::atomic<int> fwd_dyn{1};         // dynamic item queue: 0 never, 1 varlen only, 2 every persistent launch
    std::atomic<int> fwd_xcdq{1};        // dynamic queue kind: 1 one unit-major queue per XCD, 0 one global
                                         // heaviest-row-block-first queue
    std::atomic<int> fwd_pipe{1};        // software-pipelined loop over the unmasked key tiles
    std::atomic<int> fwd_decode{1};      // split-KV decode kernel when seqlen_q * H/Hk <= 32
    std::atomic<int> dec_wg_per_cu{2};   // decode split target: workgroups per CU over all (b, kv head)
    std::atomic<int> dec_mr{16};         // decode MFMA rows: 16 when the query rows fit 16 (C5: 105 vs
                                         // 110 us with dec_hmaj = 1), else 32
    std::atomic<int> comb_row{1};        // split combine: one workgroup per row when rows are few
    std::atomic<int> dec_fold{0};        // decode: the last split of each (b, kv head) merges the partials
    std::atomic<int> dec_bal{1};         // decode over per-sequence cache lengths (2 <= b <= 64): split
                                         // slots shared in proportion to the key tiles (ragged caches)
                                         // (no separate combine launch; C5: 126.8 vs 105.5 us - the
                                         // coherent partial stores and the 64-wave merge tail cost
                                         // more than the 5 us combine launch they replace)
    std::atomic<int> bwd_order{0};       // backward grid: 1 = the key blocks of one (b, kv head) consecutive
                                         // on one XCD (they then sweep the same Q / dO tiles together;
                                         // C3: 3.03 vs 2.88 ms - their dQ atomics then collide)
    std::atomic<int> bwd_desc{1};        // backward query-tile sweep: 1 = last tile first (C3 on the
                                         // round-3 session-2 kernel: 2.496 vs 2.513 ms, non-causal
                                         // 4.410 vs 4.423; dK/dV equal up to fp32 summation order)
    std::atomic<int> dec_hmaj{1};        // decode workgroup: 0 = 1 kv head x 4 splits, 1 = 4 kv heads x one
                                         // split, 2 = 8 kv heads x one split (C5 fp8: 116 / 110 / 112 us)
};
Options& options();

// Records which forward kernel (and schedule) a launch used, for fmha_last_kernel(): the name,
// the persistent mode (0 = one workgroup per item, 1 boustrophedon, 2 XCD-grouped pairs,
// 3 dynamic queue), the per-XCD queues flag and the grid.  Thread-local, set by the launchers.
void note_launch(const char* kernel, int persistent, int xcdq, unsigned gx, unsigned gy, unsigned gz, int block);

// Forward for head dim bucket HD (64 or 128) and dtype; launches the combine when
// p.num_splits > 1.  Returns the launch status.
hipError_t launch_fwd_hd64_bf16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd64_f16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd128_bf16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd128_f16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd256_bf16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd256_f16(const FwdParams& p, hipStream_t st);

// Backward (preprocess + main + convert) for head dim bucket HD.
hipError_t launch_bwd_hd64_bf16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd64_f16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd128_bf16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd128_f16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd256_bf16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd256_f16(const BwdParams& p, hipStream_t st);

// fp8 (e4m3fn) Q/K/V forward, D = 128 (fmha_fwd_fp8.hip): bf16 or fp16 output.
hipError_t launch_fwd_fp8(const FwdParams& p, bool out_fp16, hipStream_t st);
// return_softmax with dropout: the dropped-out softmax [b, h, sq_r, sk_r] (fmha_sdmask_kernel.h)
hipError_t launch_sdmask_bf16(const FwdParams& p, void* s, int sq_r, int sk_r, hipStream_t st);
hipError_t launch_sdmask_f16(const FwdParams& p, void* s, int sq_r, int sk_r, hipStream_t st);

// KV-cache append (+ rotary) pass, fmha_append.hip
struct AppendParams {
    const void* q; void* q_out;
    void* kcache; void* vcache;
    const void* knew; const void* vnew;
    const int* block_table; int bt_stride; int page;
    const int* cache_seqlens; int* seqlens_out;
    const void* cos; const void* sin; int rdim; int interleaved; int q_per_token;
    int b, sq, h, hk, d, snew;
    int64_t q_batch, q_row, q_head;          // elements (q and q_out share the layout)
    int64_t kn_batch, kn_row, kn_head;       // elements (knew / vnew share the layout)
    int64_t page_stride, row_stride, head_stride;   // cache strides (elements)
};
hipError_t launch_append(const AppendParams& p, bool fp16, hipStream_t st);

// Causal ALiBi LSE convention (fmha_append.hip): the kernels bias a causal score by
// -slope |pos + diag - key| (its largest value 0 sits on the diagonal, which the in-loop
// reference max needs), the reference by +slope key (mask_hip.h:163-164); the two differ by the
// row constant slope (pos + diag), diag = sk - sq per sequence.  dst[row] = src[row] +
// sign * slope (pos + diag) for finite entries: sign +1 turns the kernels' LSE into the
// reference's (forward), -1 back (backward input).
struct LseAlibiParams {
    const float* src;
    float* dst;
    float sign;
    const float* alibi;
    int alibi_bstride;
    int b, h, seqlen_q, seqlen_k;
    const int* cu_seqlens_q;
    const int* cu_seqlens_k;
    const int* seqused_k;
    const int* leftpad_k;
    int64_t lse_batch, lse_head;
};
hipError_t launch_lse_alibi(const LseAlibiParams& p, hipStream_t st);

// D = 256 (bucket of 129..256): 4 waves x 32 rows, one wave per SIMD (512 registers:
// Q fragments and the O accumulator alone are 192), no LDS-DMA pipeline
inline int fwd_block_m(int d, int waves) { return d > 128 ? 128 : waves * 32; }
inline int fwd_num_m_blocks(int seqlen_q, int group, int d, int waves) {
    return (seqlen_q * group + fwd_block_m(d, waves) - 1) / fwd_block_m(d, waves);
}

}  // namespace xfa

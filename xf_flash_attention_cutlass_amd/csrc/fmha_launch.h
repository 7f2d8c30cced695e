// fmha_launch.h — internal host-side launch interface (one object file per head dim x dtype).
// Replaces the reference's template fan-out run_mha_fwd_splitkv_dispatch / run_flash_splitkv_fwd
// (flash_fwd_launch_template_hip.h:106-189) and the bwd launch template
// (flash_bwd_launch_template_hip.h:76-136).
#pragma once

#include "fmha_common.h"

namespace xfa {

// Tuning knobs, settable through fmha_set_option() (used for in-process A/B runs).
struct Options {
    int fwd_waves = 8;        // waves per forward workgroup (4 or 8); 32 query rows per wave
    int fwd_prio = 0;         // static s_setprio 1 for the younger half of the workgroup
    int fwd_pp = 0;           // 1: ping-pong forward schedule (8 waves, fmha_fwd_pp_kernel.h)
    int fwd_sched = 0;        // sched_group_barrier interleave bits (experiment knob)
    int fwd_store8 = 0;       // legacy 8-byte O stores (A/B knob)
    int fwd_persistent = 1;   // persistent grid (workgroups per CU; 0 = one workgroup per item)
    int fwd_slack = 8;        // deferred rescale: running max may lag by this many log2 units
    int fwd_order = 1;        // persistent item order: 0 boustrophedon, 1 XCD-grouped pairs
    int fwd_dyn = 1;          // dynamic item queue: 0 never, 1 varlen only, 2 every persistent launch
    int fwd_xcdq = 1;         // dynamic queue kind: 1 one unit-major queue per XCD, 0 one global
                              // heaviest-row-block-first queue
    int fwd_pipe = 1;         // software-pipelined loop over the unmasked key tiles
    int fwd_dbg = 0;          // timing experiments only (results invalid when set)
    int fwd_decode = 1;       // split-KV decode kernel when seqlen_q * H/Hk <= 32
    int bwd_prio = 0;         // backward: static s_setprio 1 for the younger half (A/B)
    int dec_wg_per_cu = 2;    // decode split target: workgroups per CU over all (b, kv head)
    int fwd_decode16 = 0;     // 16x16x32 decode tile when seqlen_q * H/Hk <= 16 (slower on C5: A/B knob)
    int num_cus = 256;        // filled by the C ABI from the device
};
Options& options();

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

// D = 256 (bucket of 129..256): 4 waves x 32 rows, one wave per SIMD (512 registers:
// Q fragments and the O accumulator alone are 192), no LDS-DMA pipeline
inline int fwd_block_m(int d) {
    if (d > 128) return 128;
    return options().fwd_pp ? 256 : options().fwd_waves * 32;
}
inline int fwd_num_m_blocks(int seqlen_q, int group, int d) {
    return (seqlen_q * group + fwd_block_m(d) - 1) / fwd_block_m(d);
}

}  // namespace xfa

// fmha_launch.h — internal host-side launch interface (one object file per head dim x dtype).
// Replaces the reference's template fan-out run_mha_fwd_splitkv_dispatch / run_flash_splitkv_fwd
// (flash_fwd_launch_template_hip.h:106-189) and the bwd launch template
// (flash_bwd_launch_template_hip.h:76-136).
#pragma once

#include "fmha_common.h"

namespace xfa {

constexpr int kFwdWaves = 4;                 // waves per forward workgroup
constexpr int kFwdBlockM = kFwdWaves * 32;   // query rows per forward workgroup

// Forward for head dim bucket HD (64 or 128) and dtype; launches the combine when
// p.num_splits > 1.  Returns the launch status.
hipError_t launch_fwd_hd64_bf16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd64_f16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd128_bf16(const FwdParams& p, hipStream_t st);
hipError_t launch_fwd_hd128_f16(const FwdParams& p, hipStream_t st);

// Backward (preprocess + main + convert) for head dim bucket HD.
hipError_t launch_bwd_hd64_bf16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd64_f16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd128_bf16(const BwdParams& p, hipStream_t st);
hipError_t launch_bwd_hd128_f16(const BwdParams& p, hipStream_t st);

inline int fwd_num_m_blocks(int seqlen_q, int group) {
    return (seqlen_q * group + kFwdBlockM - 1) / kFwdBlockM;
}

}  // namespace xfa

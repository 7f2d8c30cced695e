// fmha_bwd.hip — backward instantiations for one (head dim, dtype) pair (see fmha_fwd.hip).
// Launch sequence replaces run_flash_bwd_seqk_parallel (flash_bwd_launch_template_hip.h:76-136):
// preprocess (D = rowsum(dO*O), zero dQaccum) -> main (dK, dV, dQaccum) -> convert dQ.
#include "fmha_bwd_kernel.h"
#include "fmha_launch.h"

#define XFA_CAT2(a, b) a##b
#define XFA_CAT(a, b) XFA_CAT2(a, b)
#define XFA_FN(hd, dt) XFA_CAT(XFA_CAT(XFA_CAT(launch_bwd_hd, hd), _), dt)

namespace xfa {

#if XFA_DT_BF16
typedef __bf16 elem_t;
#else
typedef _Float16 elem_t;
#endif

template <int HD, typename T>
static hipError_t launch_bwd_impl(const BwdParams& p, hipStream_t st) {
    const int64_t tokens = p.cu_seqlens_q ? (p.acc_head / p.acc_row) : (int64_t)p.b * p.seqlen_q;
    const int total_rows = (int)(tokens * p.h);
    const int64_t threads = (int64_t)total_rows * (HD / 8);
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    hipLaunchKernelGGL((fmha_bwd_pre_kernel<HD, T>), dim3(blocks), dim3(256), 0, st, p, total_rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;

    const bool mask = p.wl >= 0 || p.wr >= 0;
    const bool feat = p.alibi || p.softcap_on || p.cu_seqlens_q || p.cu_seqlens_k || p.drop;
    // [mask][feat][deterministic slices] (D > 128: one deterministic instance, MASK = FEAT = true)
    constexpr bool R = bwd_rmw<HD>();
    void (*const kerns[2][2][2])(const BwdParams) = {
        {{fmha_bwd_kernel<HD, T, false, false>, fmha_bwd_kernel<HD, T, !R, !R, true>},
         {fmha_bwd_kernel<HD, T, false, true>, fmha_bwd_kernel<HD, T, !R, true, true>}},
        {{fmha_bwd_kernel<HD, T, true, false>, fmha_bwd_kernel<HD, T, true, !R, true>},
         {fmha_bwd_kernel<HD, T, true, true>, fmha_bwd_kernel<HD, T, true, true, true>}}};
    void (*kern)(const BwdParams) = kerns[mask][feat][p.dq_slices ? 1 : 0];
    const size_t smem = bwd_smem_bytes<HD>();
    static std::atomic<unsigned long long> attr_done{0};
    once_per_device(attr_done, p.device, [&] {
        for (int i = 0; i < 8; ++i)
            (void)hipFuncSetAttribute((const void*)kerns[i >> 2][(i >> 1) & 1][i & 1],
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    });
    const int nkb = (p.seqlen_k + bwd_block_n<HD>() - 1) / bwd_block_n<HD>();
    BwdParams pp = p;
    pp.order = !p.dq_slices && p.order && (p.b * p.hk) % 8 == 0;
    // deterministic: one workgroup per (batch x kv head, dQ slice), walking its key blocks
    const dim3 grid = p.dq_slices ? dim3(p.b * p.hk, p.dq_slices)
                    : pp.order ? dim3(p.b * p.hk * nkb) : dim3(p.b * p.hk, nkb);
    hipLaunchKernelGGL(kern, grid, dim3(bwd_waves<HD>() * 64), smem, st, pp);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((fmha_bwd_convert_kernel<HD, T>), dim3(blocks), dim3(256), 0, st, p, total_rows);
    return hipGetLastError();
}

hipError_t XFA_FN(XFA_HD, XFA_DTN)(const BwdParams& p, hipStream_t st) {
    return launch_bwd_impl<XFA_HD, elem_t>(p, st);
}

}  // namespace xfa

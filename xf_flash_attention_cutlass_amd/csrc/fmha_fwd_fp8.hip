// fmha_fwd_fp8.hip — launches of the fp8 (e4m3fn) Q/K/V forward (fmha_fwd_fp8_kernel.h), D = 128,
// bf16 or fp16 output; persistent XCD-paired grid as the bf16 forward.
#include "fmha_fwd_fp8_kernel.h"
#include "fmha_fwd8w_kernel.h"
#if XFA_VARIANTS
#include "fmha_fwd8pp_kernel.h"   // (fp8_w4 = 2: the variants build only, build.py --variants)
#endif
#include "fmha_launch.h"

namespace xfa {

// 4-wave fp8 forward (fmha_fwd8w_kernel.h): no left window (the 8-wave kernel's masked loop
// handles those)
template <bool F16>
static hipError_t launch_fp8_w4(const FwdParams& p, hipStream_t st) {
    const int n_mb = (p.seqlen_q * p.group + kFwd8wRows - 1) / kFwd8wRows;
    FwdParams pp = p;
    pp.n_mblocks = n_mb;
    pp.persistent = 0;
    dim3 grid(p.b * p.hk, n_mb, 1);
    const int items = p.b * p.hk * n_mb;
    if (p.persist_per_cu > 0 && items > p.num_cus) {
        pp.persistent = p.work_ctr ? 3 : (p.order == 1 && p.num_cus % 8 == 0) ? 2 : 1;
        pp.xcd_queues = p.work_ctr && p.xcdq && p.num_cus % 8 == 0 && p.b * p.hk >= 8;
        grid = dim3(p.num_cus, 1, 1);
    }
    static std::atomic<unsigned long long> attr_done{0};
    once_per_device(attr_done, p.device, [&] { (void)hipFuncSetAttribute((const void*)fmha_fwd8w_kernel<F16>, hipFuncAttributeMaxDynamicSharedMemorySize, kFwd8wSmem); });
    note_launch("fmha_fwd8w_kernel", pp.persistent, pp.xcd_queues, grid.x, grid.y, grid.z, 256);
    hipLaunchKernelGGL((fmha_fwd8w_kernel<F16>), grid, dim3(256), kFwd8wSmem, st, pp);
    return hipGetLastError();
}

#if XFA_VARIANTS
// 8-wave ping-pong fp8 forward (fmha_fwd8pp_kernel.h): the same items, schedules, eligibility
template <bool F16>
static hipError_t launch_fp8_pp(const FwdParams& p, hipStream_t st) {
    const int n_mb = (p.seqlen_q * p.group + kFwd8ppRows - 1) / kFwd8ppRows;
    FwdParams pp = p;
    pp.n_mblocks = n_mb;
    pp.persistent = 0;
    dim3 grid(p.b * p.hk, n_mb, 1);
    const int items = p.b * p.hk * n_mb;
    if (p.persist_per_cu > 0 && items > p.num_cus) {
        pp.persistent = p.work_ctr ? 3 : (p.order == 1 && p.num_cus % 8 == 0) ? 2 : 1;
        pp.xcd_queues = p.work_ctr && p.xcdq && p.num_cus % 8 == 0 && p.b * p.hk >= 8;
        grid = dim3(p.num_cus, 1, 1);
    }
    static std::atomic<unsigned long long> attr_done{0};
    once_per_device(attr_done, p.device, [&] { (void)hipFuncSetAttribute((const void*)fmha_fwd8pp_kernel<F16>, hipFuncAttributeMaxDynamicSharedMemorySize, kFwd8ppSmem); });
    note_launch("fmha_fwd8pp_kernel", pp.persistent, pp.xcd_queues, grid.x, grid.y, grid.z, 512);
    hipLaunchKernelGGL((fmha_fwd8pp_kernel<F16>), grid, dim3(512), kFwd8ppSmem, st, pp);
    return hipGetLastError();
}
#endif

template <typename T>
static hipError_t launch_fp8_t(const FwdParams& p, hipStream_t st) {
    constexpr int NW = 8;
    const bool mask = p.wl >= 0 || p.wr >= 0;
    const int rows = p.seqlen_q * p.group;
    const int n_mb = (rows + NW * 32 - 1) / (NW * 32);
    dim3 grid(p.b * p.hk, n_mb, 1);
    FwdParams pp = p;
    pp.n_mblocks = n_mb;
    pp.persistent = 0;
    if (p.persist_per_cu > 0) {
        const int items = p.b * p.hk * n_mb;
        const int slots = p.num_cus * p.persist_per_cu;
        if (items > slots) {
            pp.persistent = (p.order == 1 && slots % 8 == 0) ? 2 : 1;
            grid = dim3(slots, 1, 1);
        }
    }
    const size_t smem = 8 * (size_t)kFp8Tile;     // K and V, four buffers each
    void (*kern)(const FwdParams) = mask ? fmha_fwd_fp8_kernel<T, NW, true> : fmha_fwd_fp8_kernel<T, NW, false>;
    static std::atomic<unsigned long long> attr_done{0};
    once_per_device(attr_done, p.device, [&] {
        (void)hipFuncSetAttribute((const void*)fmha_fwd_fp8_kernel<T, NW, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        (void)hipFuncSetAttribute((const void*)fmha_fwd_fp8_kernel<T, NW, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    });
    note_launch("fmha_fwd_fp8_kernel<8 waves>", pp.persistent, 0, grid.x, grid.y, grid.z, NW * 64);
    hipLaunchKernelGGL(kern, grid, dim3(NW * 64), smem, st, pp);
    return hipGetLastError();
}

hipError_t launch_fwd_fp8(const FwdParams& p, bool out_fp16, hipStream_t st) {
#if XFA_VARIANTS
    if (p.fwd4 == 2 && p.k_row == p.v_row && (p.wl < 0 || p.wl >= p.seqlen_k))
        return out_fp16 ? launch_fp8_pp<true>(p, st) : launch_fp8_pp<false>(p, st);
#endif
    if (p.fwd4 && p.k_row == p.v_row && (p.wl < 0 || p.wl >= p.seqlen_k))
        return out_fp16 ? launch_fp8_w4<true>(p, st) : launch_fp8_w4<false>(p, st);
    return out_fp16 ? launch_fp8_t<_Float16>(p, st) : launch_fp8_t<__bf16>(p, st);
}

}  // namespace xfa

#ifdef XFA_FWD8_STAMPS
// diagnostic builds only: copy out (and optionally clear) the 4-wave fp8 phase stamps
extern "C" int fmha_fwd8_stamps(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(xfa::g_fwd8_stamps), sizeof(xfa::g_fwd8_stamps)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long zero[4 * 8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(xfa::g_fwd8_stamps), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// fmha_fwd.hip — forward instantiations for one (head dim, dtype) pair.
// Compiled once per pair with -DXFA_HD=<64|128|256> -DXFA_DT=<bf16|f16> (see build.py), which
// keeps the per-variant kernels in separate code objects (co-compiled template variants
// perturb each other's register allocation, cdna_hip_programming.md §5.4 rule 19).
#include "fmha_fwd_kernel.h"
#if XFA_HD == 128
#if XFA_VARIANTS && XFA_HD == 128
#include "fmha_fwd4_kernel.h"     // (fwd_w4 = 1: the variants build only, build.py --variants)
#endif
#include "fmha_fwdpp_kernel.h"
#endif
#include "fmha_decode_kernel.h"
#include "fmha_sdmask_kernel.h"
#include "fmha_launch.h"

#ifndef XFA_HD
#error "XFA_HD must be defined"
#endif

#define XFA_CAT2(a, b) a##b
#define XFA_CAT(a, b) XFA_CAT2(a, b)
#define XFA_FN(hd, dt) XFA_CAT(XFA_CAT(XFA_CAT(launch_fwd_hd, hd), _), dt)

namespace xfa {

#if XFA_DT_BF16
typedef __bf16 elem_t;
#else
typedef _Float16 elem_t;
#endif

static hipError_t launch_combine(const FwdParams& p, int hd, hipStream_t st,
                                 void (*kern)(const CombineParams),
                                 void (*row_kern)(const CombineParams) = nullptr) {
    CombineParams cp;
    cp.oaccum = p.oaccum;
    cp.lseaccum = p.lseaccum;
    cp.o = p.o;
    cp.lse = p.lse;
    cp.o_batch = p.o_batch; cp.o_row = p.o_row; cp.o_head = p.o_head;
    cp.lse_batch = p.lse_batch; cp.lse_head = p.lse_head;
    cp.b = p.b; cp.h = p.h; cp.seqlen_q = p.seqlen_q; cp.d = p.d; cp.hd = hd;
    cp.num_splits = p.num_splits;
    cp.dec_ns = p.decode && p.dec_bal ? p.dec_ns : nullptr;
    const int64_t crow = (int64_t)p.b * p.h * p.seqlen_q;
    const int ext = cp.dec_ns ? p.dec_cap : p.num_splits;
    // few rows (the decode shapes): one workgroup per row, all of its partials in flight at once
    if (row_kern && p.comb_row && ext <= 128 && crow <= 8 * (int64_t)p.num_cus) {
        hipLaunchKernelGGL(row_kern, dim3((unsigned)crow), dim3(256), 0, st, cp);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)((crow + 3) / 4)), dim3(256), 0, st, cp);
    return hipGetLastError();
}

template <int HD, typename T>
static hipError_t launch_decode(const FwdParams& p, hipStream_t st) {
    hipError_t e;
    if (p.dec_hmaj == 2) {
        // 8 waves = the 8 kv heads of one split: one cache row's heads are read side by side
        constexpr int NWV = 2 * kDecWaves;
        const size_t smem = (size_t)NWV * 2 * kDecKeys * HD * 2;
        static std::atomic<unsigned long long> attr_done{0};
        once_per_device(attr_done, p.device, [&] {
            (void)hipFuncSetAttribute((const void*)fmha_decode_kernel<HD, T, true, 32, NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            (void)hipFuncSetAttribute((const void*)fmha_decode_kernel<HD, T, false, 32, NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            (void)hipFuncSetAttribute((const void*)fmha_decode_kernel<HD, T, true, 16, NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            (void)hipFuncSetAttribute((const void*)fmha_decode_kernel<HD, T, false, 16, NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        });
        const dim3 grid(p.b * p.hk / NWV, p.num_splits);
        note_launch(p.dec_mr == 16 ? "fmha_decode_kernel<16 rows, 8 heads>" : "fmha_decode_kernel<32 rows, 8 heads>", 0, 0, grid.x, grid.y, grid.z, NWV * 64);
        if (p.dec_mr == 16) {
            if (p.kv_fp8) hipLaunchKernelGGL((fmha_decode_kernel<HD, T, true, 16, NWV>), grid, dim3(NWV * 64), smem, st, p);
            else hipLaunchKernelGGL((fmha_decode_kernel<HD, T, false, 16, NWV>), grid, dim3(NWV * 64), smem, st, p);
        } else {
            if (p.kv_fp8) hipLaunchKernelGGL((fmha_decode_kernel<HD, T, true, 32, NWV>), grid, dim3(NWV * 64), smem, st, p);
            else hipLaunchKernelGGL((fmha_decode_kernel<HD, T, false, 32, NWV>), grid, dim3(NWV * 64), smem, st, p);
        }
    } else {
        const size_t smem = (size_t)kDecWaves * 2 * kDecKeys * HD * 2;
        const dim3 grid = p.dec_hmaj ? dim3(p.b * p.hk / kDecWaves, p.num_splits) : dim3(p.b * p.hk, p.num_splits / kDecWaves);
        note_launch(p.dec_mr == 16 ? "fmha_decode_kernel<16 rows>" : "fmha_decode_kernel<32 rows>", 0, 0, grid.x, grid.y, grid.z, kDecWaves * 64);
        if (p.dec_mr == 16) {
            if (p.kv_fp8) hipLaunchKernelGGL((fmha_decode_kernel<HD, T, true, 16>), grid, dim3(kDecWaves * 64), smem, st, p);
            else hipLaunchKernelGGL((fmha_decode_kernel<HD, T, false, 16>), grid, dim3(kDecWaves * 64), smem, st, p);
        } else {
            if (p.kv_fp8) hipLaunchKernelGGL((fmha_decode_kernel<HD, T, true, 32>), grid, dim3(kDecWaves * 64), smem, st, p);
            else hipLaunchKernelGGL((fmha_decode_kernel<HD, T, false, 32>), grid, dim3(kDecWaves * 64), smem, st, p);
        }
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (p.dec_ctr) return hipSuccess;          // the last split of each (b, kv head) merged
    return launch_combine(p, HD, st, fmha_combine_kernel<HD, T>,
                          (HD == 64 || HD == 128 || HD == 256) ? fmha_combine_row_kernel<HD, T> : nullptr);
}

template <int HD, typename T, int NW>
static hipError_t launch_fwd_nw(const FwdParams& p, hipStream_t st) {
    const bool mask = p.wl >= 0 || p.wr >= 0;
    // FEAT: per-score transforms (ALiBi, softcap) and the paged / fp8 staging paths
    const bool feat = p.alibi || p.softcap_pre > 0.f || p.block_table || p.kv_fp8 || p.drop;
    const int rows = p.seqlen_q * p.group;
    const int n_mb = (rows + NW * 32 - 1) / (NW * 32);
    dim3 grid(p.b * p.hk, n_mb, p.num_splits > 1 ? p.num_splits : 1);
    FwdParams pp = p;
    pp.n_mblocks = n_mb;
    pp.persistent = 0;
    if (p.persist_per_cu > 0) {
        const int items = p.b * p.hk * n_mb;
        const int slots = p.num_cus * p.persist_per_cu;
        if (items > slots) {
            pp.persistent = p.work_ctr ? 3 : (p.order == 1 && slots % 8 == 0) ? 2 : 1;
            pp.xcd_queues = p.work_ctr && p.xcdq && slots % 8 == 0 && p.b * p.hk >= 8;
            grid = dim3(slots, 1, grid.z);
        }
    }
    const size_t smem = (size_t)(fwd_nbuf(HD) * 2 * kBlockN * HD * 2);
    void (*kern)(const FwdParams) =
        mask ? (feat ? fmha_fwd_kernel<HD, T, NW, true, true> : fmha_fwd_kernel<HD, T, NW, true, false>)
             : (feat ? fmha_fwd_kernel<HD, T, NW, false, true> : fmha_fwd_kernel<HD, T, NW, false, false>);
    static std::atomic<unsigned long long> attr_done{0};
    once_per_device(attr_done, p.device, [&] {
        (void)hipFuncSetAttribute((const void*)fmha_fwd_kernel<HD, T, NW, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        (void)hipFuncSetAttribute((const void*)fmha_fwd_kernel<HD, T, NW, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        (void)hipFuncSetAttribute((const void*)fmha_fwd_kernel<HD, T, NW, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        (void)hipFuncSetAttribute((const void*)fmha_fwd_kernel<HD, T, NW, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    });
    note_launch(NW == 8 ? "fmha_fwd_kernel<8 waves>" : "fmha_fwd_kernel<4 waves>", pp.persistent, pp.xcd_queues, grid.x, grid.y, grid.z, NW * 64);
    hipLaunchKernelGGL(kern, grid, dim3(NW * 64), smem, st, pp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || p.num_splits <= 1) return e;
    return launch_combine(p, HD, st, fmha_combine_kernel<HD, T>,
                          (HD == 64 || HD == 128 || HD == 256) ? fmha_combine_row_kernel<HD, T> : nullptr);
}

#if XFA_HD == 128
// 4-wave / ping-pong forwards: dense / varlen, D = 128, one split, no paged / fp8 K/V /
// leftpad / dropout (those run the 8-wave kernel)
// (ALiBi, softcap and left windows: the 32x32x16 ping-pong kernel only, its score-feature pass
// and two-sided key window)
// paged K/V on the ping-pong kernel (its 32x32x16 body): every 8-row block of a 64-key tile must
// lie in one page (a power-of-two page size >= 8) and K and V must share their strides
static bool fwdpp_paged_ok(const FwdParams& p) {
    return p.page_size >= 8 && (p.page_size & (p.page_size - 1)) == 0 && p.k_batch == p.v_batch &&
           (p.fwd4 == 2 || p.fwd4 == 4);
}

static bool fwd4_eligible(const FwdParams& p) {
    const bool feat = p.alibi || p.softcap_pre > 0.f || (p.wl >= 0 && p.wl < p.seqlen_k);
    return p.fwd4 && p.d == 128 && p.k_row == p.v_row && p.num_splits <= 1 &&
           (!p.block_table || fwdpp_paged_ok(p)) && !p.kv_fp8 && !p.leftpad_k && !p.drop &&
           (!feat || p.fwd4 == 2 || p.fwd4 == 4);
}

// 8-wave ping-pong forward (fmha_fwdpp_kernel.h): the same items, schedules and eligibility
static hipError_t launch_fwdpp(const FwdParams& p, hipStream_t st) {
    const int n_mb = (p.seqlen_q * p.group + kFwdppRows - 1) / kFwdppRows;
    FwdParams pp = p;
    pp.n_mblocks = n_mb;
    pp.persistent = 0;
    dim3 grid(p.b * p.hk, n_mb, 1);
    const int items = p.b * p.hk * n_mb;
    const int slots = p.num_cus;
    if (p.persist_per_cu > 0 && items > slots) {
        pp.persistent = p.work_ctr ? 3 : (p.order == 1 && slots % 8 == 0) ? 2 : 1;
        pp.xcd_queues = p.work_ctr && p.xcdq && slots % 8 == 0 && p.b * p.hk >= 8;
        grid = dim3(slots, 1, 1);
    }
    constexpr bool BF = std::is_same<elem_t, __bf16>::value;
    // fwd_w4 = 3: the body on the 16x16x32 MFMA shape (tools/gen_fwdpp16.py); 4 (auto, the
    // default): 16x16x32 where no row has a right window (causal / local rows: 32x32x16), the
    // faster of the two per mask on the same box
    const bool m16 = !p.block_table &&
                     (p.fwd4 == 3 || (p.fwd4 == 4 && p.wr < 0 && !p.alibi && !(p.softcap_pre > 0.f)));
    static std::atomic<unsigned long long> attr_done{0};
    once_per_device(attr_done, p.device, [&] {
        (void)hipFuncSetAttribute((const void*)fmha_fwdpp_kernel<BF, false>, hipFuncAttributeMaxDynamicSharedMemorySize, kFwdppSmem);
        (void)hipFuncSetAttribute((const void*)fmha_fwdpp_kernel<BF, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kFwdppSmem);
        (void)hipFuncSetAttribute((const void*)fmha_fwdpp_kernel<BF, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kFwdppSmem);
    });
    note_launch(m16 ? "fmha_fwdpp16_kernel" : p.block_table ? "fmha_fwdpp_paged_kernel" : "fmha_fwdpp_kernel",
                pp.persistent, pp.xcd_queues, grid.x, grid.y, grid.z, 512);
    if (m16) hipLaunchKernelGGL((fmha_fwdpp_kernel<BF, true>), grid, dim3(512), kFwdppSmem, st, pp);
    else if (p.block_table) hipLaunchKernelGGL((fmha_fwdpp_kernel<BF, false, true>), grid, dim3(512), kFwdppSmem, st, pp);
    else hipLaunchKernelGGL((fmha_fwdpp_kernel<BF, false>), grid, dim3(512), kFwdppSmem, st, pp);
    return hipGetLastError();
}

static hipError_t launch_fwd4(const FwdParams& p, hipStream_t st) {
    if (p.fwd4 >= 2) return launch_fwdpp(p, st);
#if !XFA_VARIANTS
    return hipErrorNotSupported;   // (fmha_set_option refuses fwd_w4 = 1 in this build)
#else
    const int n_mb = (p.seqlen_q * p.group + kFwd4Rows - 1) / kFwd4Rows;
    FwdParams pp = p;
    pp.n_mblocks = n_mb;
    pp.persistent = 0;
    dim3 grid(p.b * p.hk, n_mb, 1);
    const int items = p.b * p.hk * n_mb;
    const int slots = p.num_cus;
    if (p.persist_per_cu > 0 && items > slots) {
        pp.persistent = p.work_ctr ? 3 : (p.order == 1 && slots % 8 == 0) ? 2 : 1;
        pp.xcd_queues = p.work_ctr && p.xcdq && slots % 8 == 0 && p.b * p.hk >= 8;
        grid = dim3(slots, 1, 1);
    }
    constexpr bool BF = std::is_same<elem_t, __bf16>::value;
    static std::atomic<unsigned long long> attr_done{0};
    once_per_device(attr_done, p.device, [&] { (void)hipFuncSetAttribute((const void*)fmha_fwd4_kernel<BF>, hipFuncAttributeMaxDynamicSharedMemorySize, kFwd4Smem); });
    note_launch("fmha_fwd4_kernel", pp.persistent, pp.xcd_queues, grid.x, grid.y, grid.z, 256);
    hipLaunchKernelGGL((fmha_fwd4_kernel<BF>), grid, dim3(256), kFwd4Smem, st, pp);
    return hipGetLastError();
#endif
}
#endif

#if XFA_HD == 128
// return_softmax with dropout (fmha_sdmask_kernel.h): s [b, h, sq_r, sk_r] in the q dtype
hipError_t XFA_CAT(launch_sdmask_, XFA_DTN)(const FwdParams& p, void* s, int sq_r, int sk_r, hipStream_t st) {
    const int64_t s_head = (int64_t)sq_r * sk_r;
    hipLaunchKernelGGL((fmha_sdmask_kernel<elem_t>), dim3(p.b * p.h, sq_r), dim3(256), 0, st, p,
                       reinterpret_cast<elem_t*>(s), s_head * p.h, s_head, sk_r);
    return hipGetLastError();
}
#endif

hipError_t XFA_FN(XFA_HD, XFA_DTN)(const FwdParams& p, hipStream_t st) {
#if XFA_HD > 128
    // D = 256: 4-wave register-staged kernel only (no decode / DMA pipeline)
    return launch_fwd_nw<XFA_HD, elem_t, 4>(p, st);
#else
    if (p.decode) return launch_decode<XFA_HD, elem_t>(p, st);
#if XFA_HD == 128
    if (fwd4_eligible(p)) return launch_fwd4(p, st);
#endif
    if (p.waves == 8) return launch_fwd_nw<XFA_HD, elem_t, 8>(p, st);
    return launch_fwd_nw<XFA_HD, elem_t, 4>(p, st);
#endif
}

}  // namespace xfa

#if defined(XFA_FWDPP_STAMPS) && XFA_HD == 128 && XFA_DT_BF16
// diagnostic builds only: copy out (and optionally clear) the ping-pong phase stamps
extern "C" int fmha_fwdpp_stamps(unsigned* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(xfa::g_fwdpp_stamps), sizeof(xfa::g_fwdpp_stamps)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned zero[8 * 8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(xfa::g_fwdpp_stamps), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

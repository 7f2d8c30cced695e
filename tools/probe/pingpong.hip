// pingpong.hip — PROBE, not product code: the 8-wave ping-pong D = 128
// forward of tools/gen_pingpong.py, dense bf16, non-causal, persistent over XCD-grouped items
// like fmha_fwd4_kernel.h.  Built by tools/probe/build.sh into tools/probe/libpingpong.so and
// timed beside the product's 4-wave kernel by tools/pingpong_ab.py.
#include "../../xf_flash_attention_cutlass_amd/csrc/fmha_common.h"
#ifndef PP_BODY
#define PP_BODY "pingpong_body.h"
#endif
#include PP_BODY

using namespace xfa;

namespace {

constexpr int kRows = 256;                 // query rows per workgroup (8 waves x 32)
constexpr int kTile = 128 * 64 * 2;
constexpr int kVReg = 4 * kTile;
constexpr int kSmem = 8 * kTile;            // 4 K + 4 V slots, 128 KiB

struct PPArgs {
    const void* q; const void* k; const void* v; void* o; float* lse;
    int b, s, h, hk;                        // [b, s, h|hk, 128] contiguous, sq == sk
    float c;                                // softmax_scale * log2(e)
    int n_mblocks;
};

__device__ __forceinline__ i32x4 srd(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
    r[3] = 0x00020000;
    return r;
}

template <bool FULL>
__device__ __forceinline__ void pp_item(const PPArgs& p, char* smem, int bh, int m_block) {
    constexpr int HD = 128;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, lr = lane & 31, hh = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bidx = bh / p.hk, hk_i = bh - bidx * p.hk;
    const int G = p.h / p.hk;
    const int sq = p.s, sk = p.s;
    const int rows_total = sq * G;
    const int row0 = m_block * kRows;
    const int q_row = p.h * HD, k_row = p.hk * HD;
    const int row = row0 + 32 * wave + lr;
    const bool ok = row < rows_total;
    const int pos = ok ? row / G : 0;
    const int head = hk_i * G + (ok ? row - pos * G : 0);
    const int qoff = ok ? (pos * q_row + head * HD) * 2 + 16 * hh : kOOB;
    const int ooff = qoff;
    const int loff = (ok && hh == 0) ? (head * sq + pos) * 4 : kOOB;
    const char* qseq = reinterpret_cast<const char*>(p.q) + (int64_t)bidx * sq * q_row * 2;
    char* oseq = reinterpret_cast<char*>(p.o) + (int64_t)bidx * sq * q_row * 2;
    const uint32_t qbytes = (uint32_t)((int64_t)sq * q_row * 2);
    const i32x4 qsrd = srd(qseq, qbytes), osrd = srd(oseq, qbytes);
    const i32x4 lsrd = srd(p.lse + (int64_t)bidx * p.h * sq, (uint32_t)(p.h * sq * 4));
    const char* kseq = reinterpret_cast<const char*>(p.k) + ((int64_t)bidx * sk * k_row + hk_i * HD) * 2;
    const char* vseq = reinterpret_cast<const char*>(p.v) + ((int64_t)bidx * sk * k_row + hk_i * HD) * 2;
    const int ntl = (sk + 63) / 64;
    const int kvbytes = ((sk - 1) * k_row + HD) * 2;
    const int kblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)kseq);
    const int kbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)kseq >> 32) & 0xFFFF);
    const int vblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)vseq);
    const int vbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)vseq >> 32) & 0xFFFF);
    // DMA: wave w loads 8-row block w of every tile, pieces i = chunks 8i..8i+7 (lane l at 16 l)
    const int r = 8 * wave + lr / 4;
    const int cch = 4 * hh + ((lane & 3) ^ ((r >> 2) & 3));
    const int dma0 = r * k_row * 2 + cch * 16;
    const int sbase = (int)(size_t)smem;
    int kb[2], vb[2];
    const int q4 = (lane & 15) >> 2;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        kb[u] = sbase + kv_off<HD>(lr, 2 * u + hh);
        const int rr = 8 * u + 4 * hh + q4;
        const int col = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        vb[u] = sbase + kVReg + kv_off<HD>(rr, col >> 3) + 8 * ((col >> 2) & 1);
    }
    const int kstep = __builtin_amdgcn_readfirstlane(64 * k_row * 2);
    const int kdst = __builtin_amdgcn_readfirstlane(sbase + wave * 2048);
    const int grp = __builtin_amdgcn_readfirstlane(wave >> 2);
    const float thr = __builtin_inff();
    if constexpr (FULL)
        pp_item_full_bf16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, grp, p.c,
                          thr, kb[0], kb[1], vb[0], vb[1], dma0, dma0 + 128, qoff, ooff, loff);
    else
        pp_item_skel_bf16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, grp, p.c,
                          thr, kb[0], kb[1], vb[0], vb[1], dma0, dma0 + 128, qoff, ooff, loff);
}

// persistent grid, one workgroup per CU, XCD-grouped (n-1-i, i) row-block pairs
template <bool FULL>
__global__ void __launch_bounds__(512, 1) pp_kernel(const PPArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nbh = p.b * p.hk;
    const int g = gridDim.x;
    for (int k = 0;; ++k) {
        const int nm = p.n_mblocks, npair = (nm + 1) >> 1;
        const int bid = (int)blockIdx.x;
        const int v = (bid & 7) * (g >> 3) + (bid >> 3);
        const int q = (k >> 1) * g + v;
        if (q >= nbh * npair) break;
        const int bh = q / npair;
        const int i = q - bh * npair;
        const int m_block = (k & 1) ? i : nm - 1 - i;
        if ((k & 1) && i == nm - 1 - i) continue;
        pp_item<FULL>(p, smem, bh, m_block);
    }
}

}  // namespace

extern "C" int pp_launch(const void* q, const void* k, const void* v, void* o, float* lse, int b, int s,
                         int h, int hk, float softmax_scale, int full, hipStream_t st) {
    if (s % 64 != 0 || h % hk != 0) return -1;
    PPArgs p{q, k, v, o, lse, b, s, h, hk, softmax_scale * 1.4426950408889634f, 0};
    p.n_mblocks = (s * (h / hk) + kRows - 1) / kRows;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus % 8) return -2;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)pp_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, kSmem);
        (void)hipFuncSetAttribute((const void*)pp_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, kSmem);
        attr = true;
    }
    if (full) hipLaunchKernelGGL(pp_kernel<true>, dim3(cus), dim3(512), kSmem, st, p);
    else hipLaunchKernelGGL(pp_kernel<false>, dim3(cus), dim3(512), kSmem, st, p);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

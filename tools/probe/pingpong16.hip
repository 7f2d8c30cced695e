// pingpong16.hip — PROBE, not product code: the 8-wave ping-pong D = 128
// forward of tools/gen_pingpong16.py (v_mfma_f32_16x16x32_bf16), otherwise as pingpong.hip.
// Built by tools/probe/build16.sh, timed beside the 32x32x16 probe by tools/pingpong_ab.py.
#include "../../xf_flash_attention_cutlass_amd/csrc/fmha_common.h"
#ifndef PP_BODY
#define PP_BODY "pingpong16_body.h"
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
    // 16x16x32 operands: lane l holds row 16 rt + (l & 15) of the wave's 32 rows, group g = l >> 4
    const int g = lane >> 4, l16 = lane & 15;
    int qoff[2], ooff[2], loff[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const int row = row0 + 32 * wave + 16 * rt + l16;
        const bool ok = row < rows_total;
        const int pos = ok ? row / G : 0;
        const int head = hk_i * G + (ok ? row - pos * G : 0);
        const int base = (pos * q_row + head * HD) * 2;
        qoff[rt] = ok ? base + 16 * g : kOOB;     // Q chunk 4 s + g (+ 64 s immediate)
        ooff[rt] = ok ? base + 8 * g : kOOB;      // O d 16 dt + 4 g (+ 32 dt immediate)
        loff[rt] = (ok && g == 0) ? (head * sq + pos) * 4 : kOOB;
    }
    (void)hh;
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
    // K row reads (A of S^T = K Q^T): key 16 kt + l16, chunk 4 s + g of the kv_off image
    const int kb0 = sbase + 2048 * ((lane >> 3) & 1) + 64 * (lane & 7) + 16 * (g ^ ((lane >> 2) & 3));
    // V^T transposed reads (A of O^T += V^T P^T): lane 4q + p of group g reads key 4 g + q
    // (+ 32 ks + 16 h), d columns 16 dt + 4 p .. +3; base per dt parity e
    const int q4 = (lane & 15) >> 2, p4 = lane & 3;
    int vb[2];
#pragma unroll
    for (int e = 0; e < 2; ++e)
        vb[e] = sbase + kVReg + 2048 * (g >> 1) + 64 * (4 * (g & 1) + q4) +
                16 * ((2 * e + (p4 >> 1)) ^ g) + 8 * (p4 & 1);
    const int kstep = __builtin_amdgcn_readfirstlane(64 * k_row * 2);
    const int kdst = __builtin_amdgcn_readfirstlane(sbase + wave * 2048);
    const int grp = __builtin_amdgcn_readfirstlane(wave >> 2);
    const float thr = __builtin_inff();
    if constexpr (FULL)
        pp16_item_full_bf16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, grp, p.c,
                            thr, kb0, vb[0], vb[1], dma0, dma0 + 128, qoff[0], qoff[1], ooff[0], ooff[1],
                            loff[0], loff[1]);
    else
        pp16_item_skel_bf16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, grp, p.c,
                            thr, kb0, vb[0], vb[1], dma0, dma0 + 128, qoff[0], qoff[1], ooff[0], ooff[1],
                            loff[0], loff[1]);
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

// fmha_fwd8w_kernel.h — 4-wave fp8 (e4m3fn) forward, D = 128 (one wave per SIMD, 64 query rows
// per wave): the structure of fmha_fwd4_kernel.h (bf16) on the block-scaled fp8 MFMA.
//
// Same semantics as fmha_fwd_fp8_kernel.h (north_star's fp8 GEMMs; the bf16 forward of the
// reference, flash_fwd_kernel_hip.h:1023-1200, on the dequantised inputs with P rounded to e4m3
// for PV).  Runs the fp8 launches with no left window (fp8_w4 knob); the item's whole
// pipeline is one generated asm statement (fmha_fwd8_body.h, tools/gen_fwd8.py) and this file
// computes its geometry: descriptors, per-lane LDS / DMA / row offsets, tile counts.
#pragma once

#include "fmha_common.h"
#ifdef XFA_FWD8_BODY                     // A/B builds of a generated variant (tools/fwd8_variant.py)
#include XFA_FWD8_BODY
#else
#include "fmha_fwd8_body.h"
#endif

namespace xfa {

#ifdef XFA_FWD8_STAMPS
// Diagnostic build only (gen_fwd8.py --stamps, read by tools/fwd8_stamps.py): each wave sums
// the s_memtime cycles per phase class in lanes 0..7 of one register; the kernel adds them into
// this array at its end (read by fmha_fwd8_stamps).
static __device__ unsigned long long g_fwd8_stamps[4 * 8];   // (64-bit: 256 workgroups x launches)
#define XFA_F8_ACC_PARAM , unsigned& acc
#define XFA_F8_ACC_ARG , acc
#else
#define XFA_F8_ACC_PARAM
#define XFA_F8_ACC_ARG
#endif

constexpr int kFwd8wRows = 256;            // query rows per workgroup (4 waves x 64)
constexpr int kFwd8wTile = 64 * 128;       // bytes of one fp8 K (or V) tile
constexpr int kFwd8wVReg = 4 * kFwd8wTile; // V ring after the 4 K slots
constexpr int kFwd8wSmem = 8 * kFwd8wTile; // 64 KiB

__device__ __forceinline__ i32x4 fwd8w_srd(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
    r[3] = 0x00020000;
    return r;
}

// fp8 LDS images (fmha_fwd_fp8_kernel.h): XOR of the 16-byte chunk by the row
__device__ __forceinline__ int k8w_off(int row, int chunk) { return row * 128 + 16 * (chunk ^ ((row >> 1) & 7)); }
// V: the transposed reads take rows 4h + {0..3, 8..11} (+ 16 kb) per lane half h (the P
// k permutation, tools/gen_fwd8.py): the chunk XOR uses row bits 1 and 3 so the 8 rows of
// one read half land on 4 different chunk pairs per row parity (conflict-free)
__device__ __forceinline__ int v8w_swz(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }
__device__ __forceinline__ int v8w_off(int row, int chunk) { return row * 128 + 16 * (chunk ^ v8w_swz(row)); }

// One (batch x kv head, 256-row query block) item.
template <bool F16>
__device__ __forceinline__ void fwd8w_item(const FwdParams& p, char* smem, const int bh, const int m_block XFA_F8_ACC_PARAM) {
    constexpr int HD = 128;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));        // item-local (see fmha_fwd4_kernel.h)
    const int lane = tid & 63;
    const int lr = lane & 31;
    const int hh = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int bidx = bh / p.hk;
    const int hk_i = bh - bidx * p.hk;
    const int sq = p.seqlen_q, sk = p.seqlen_k;
    const int G = p.group;
    const int rows_total = sq * G;
    const int row0 = m_block * kFwd8wRows;
    if (row0 >= rows_total) return;          // workgroup-uniform
    const int diag = sk - sq;
    auto lim_r = [&](int pos) { return p.wr >= 0 ? min(sk, pos + diag + p.wr + 1) : sk; };

    const int pos_hi = (min(row0 + kFwd8wRows, rows_total) - 1) / G;
    const int n_hi = sk > 0 ? lim_r(pos_hi) : 0;
    const int ntl = n_hi > 0 ? (n_hi + kBlockN - 1) / kBlockN : 0;

    const int wrow0 = row0 + 64 * wave;
    int t_w = -1, e_w = 1 << 30;
    if (wrow0 < rows_total && ntl > 0) {
        const int wp_lo = wrow0 / G, wp_hi = (min(wrow0 + 64, rows_total) - 1) / G;
        const int lr_hi = lim_r(wp_hi), lr_lo = lim_r(wp_lo);
        t_w = lr_hi > 0 ? min(ntl, (lr_hi + kBlockN - 1) / kBlockN) - 1 : -1;
        e_w = lr_lo > 0 ? lr_lo / kBlockN : 0;
    }
    t_w = __builtin_amdgcn_readfirstlane(t_w);
    e_w = __builtin_amdgcn_readfirstlane(e_w);

    int qoff[2], ooff[2], loff[2], lim[2];
    const int q_row = (int)p.q_row, q_head = (int)p.q_head;
    const int o_row = (int)p.o_row, o_head = (int)p.o_head;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
        const int row = wrow0 + 32 * rb + lr;
        const bool ok = row < rows_total;
        const int pos = ok ? row / G : 0;
        const int head = hk_i * G + (ok ? row - pos * G : 0);
        qoff[rb] = ok ? pos * q_row + head * q_head + 32 * hh : kOOB;          // fp8 bytes
        ooff[rb] = ok ? (pos * o_row + head * o_head) * 2 + 16 * hh : kOOB;
        loff[rb] = (ok && hh == 0) ? (int)(head * p.lse_head + pos) * 4 : kOOB;
        lim[rb] = (ok ? lim_r(pos) : sk) - 4 * hh;
    }

    if (ntl <= 0) {
        // no visible key for any row: O = 0, LSE = +inf (the reference's empty-row output)
        typedef __attribute__((ext_vector_type(4))) unsigned u4;
        char* oseq = reinterpret_cast<char*>(p.o) + (int64_t)bidx * p.o_batch * 2;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            if (ooff[rb] == kOOB) continue;
#pragma unroll
            for (int c = 0; c < 8; ++c) *reinterpret_cast<u4*>(oseq + ooff[rb] + 32 * c) = u4{0, 0, 0, 0};
            if (p.lse && hh == 0) p.lse[(int64_t)bidx * p.lse_batch + loff[rb] / 4] = INFINITY;
        }
        return;
    }

    const char* qseq = reinterpret_cast<const char*>(p.q) + (int64_t)bidx * p.q_batch;
    char* oseq = reinterpret_cast<char*>(p.o) + (int64_t)bidx * p.o_batch * 2;
    const uint32_t qbytes = (uint32_t)((int64_t)(sq - 1) * p.q_row + (int64_t)(p.h - 1) * p.q_head + HD);
    const uint32_t obytes = (uint32_t)(((int64_t)(sq - 1) * p.o_row + (int64_t)(p.h - 1) * p.o_head + HD) * 2);
    const i32x4 qsrd = fwd8w_srd(qseq, qbytes), osrd = fwd8w_srd(oseq, obytes);
    const float* lseq = p.lse ? p.lse + (int64_t)bidx * p.lse_batch : p.lse;
    const int64_t lbytes = p.lse ? ((int64_t)(p.h - 1) * p.lse_head + sq) * 4 : 0;
    const i32x4 lsrd = fwd8w_srd(lseq, (uint32_t)min(lbytes, (int64_t)kOOB - 1));
    const int k_row = (int)p.k_row, v_row = (int)p.v_row;
    const char* kseq = reinterpret_cast<const char*>(p.k) + (int64_t)bidx * p.k_batch + (int64_t)hk_i * p.k_head;
    const char* vseq = reinterpret_cast<const char*>(p.v) + (int64_t)bidx * p.v_batch + (int64_t)hk_i * p.v_head;
    const int nk = min(sk, ntl * kBlockN);
    const uint32_t kvbytes = (uint32_t)((nk - 1) * k_row + HD);
    const int kblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)kseq);
    const int kbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)kseq >> 32) & 0xFFFF);
    const int vblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)vseq);
    const int vbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)vseq >> 32) & 0xFFFF);

    // LDS-DMA pieces g = 2 wave + i: 8 rows x 8 chunks, lane l lands at g KiB + 16 l, fetched
    // from the source chunk the image's XOR places there (K and V images differ)
    int dk[2], dv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int g = wave * 2 + i;
        const int r = 8 * g + (lane >> 3);
        dk[i] = r * k_row + 16 * ((lane & 7) ^ ((r >> 1) & 7));
        dv[i] = r * v_row + 16 * ((lane & 7) ^ v8w_swz(r));
    }
    const int sbase = (int)(size_t)smem;
    int ka[4], va[4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) ka[2 * s + u] = sbase + k8w_off(lr, 4 * s + 2 * hh + u);
    {
        const int i = lane & 15, q = i >> 1, pb8 = i & 1, g = (lane >> 4) & 1;
        const int r = 4 * hh + (q & 3) + 8 * (q >> 2);   // read kb adds 16 kb rows
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) va[dt] = sbase + kFwd8wVReg + v8w_off(r, 2 * dt + g) + 8 * pb8;
    }
    const int kstep = __builtin_amdgcn_readfirstlane(kBlockN * k_row);
    const int kdst = __builtin_amdgcn_readfirstlane(sbase + wave * 2048);
    const float c = p.scale_log2 * p.q_scale * p.k_scale;
    const float thr = __builtin_amdgcn_exp2f(fminf(p.max_slack, 8.f));   // P <= 256 < 448
    if constexpr (F16)
        fwd8_item_f16(kblo, kbhi, vblo, vbhi, (int)kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w,
                      c, thr, p.v_scale, ka[0], ka[1], ka[2], ka[3], va[0], va[1], va[2], va[3], dk[0], dk[1],
                      dv[0], dv[1], lim[0], lim[1], qoff[0], qoff[1], ooff[0], ooff[1], loff[0], loff[1] XFA_F8_ACC_ARG);
    else
        fwd8_item_bf16(kblo, kbhi, vblo, vbhi, (int)kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w,
                       c, thr, p.v_scale, ka[0], ka[1], ka[2], ka[3], va[0], va[1], va[2], va[3], dk[0], dk[1],
                       dv[0], dv[1], lim[0], lim[1], qoff[0], qoff[1], ooff[0], ooff[1], loff[0], loff[1] XFA_F8_ACC_ARG);
}

// Persistent grid (one workgroup per CU): XCD-grouped (n-1-i, i) row-block pairs, or (fwd_dyn
// = 2) the per-XCD dynamic item queues, as the bf16 kernels.
template <bool F16>
__global__ void __launch_bounds__(256, 1) fmha_fwd8w_kernel(const FwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int s_claim[2];
    const int nbh = p.b * p.hk;
    const int g = gridDim.x;
#ifdef XFA_FWD8_STAMPS
    unsigned acc = 0;
#endif
    for (int k = 0;; ++k) {
        int bh, m_block;
        if (p.persistent == 3) {
            const int x = p.xcd_queues ? (int)(blockIdx.x & 7) : 0;
            const int nq = p.xcd_queues ? (nbh - x + 7) >> 3 : nbh;
            if (threadIdx.x == 0) s_claim[k & 1] = atomicAdd(p.work_ctr + 2 + x, 1);
            __syncthreads();
            const int q = s_claim[k & 1];
            if (q >= nq * p.n_mblocks) break;
            if (p.xcd_queues) {
                bh = x + 8 * (q / p.n_mblocks);
                m_block = p.n_mblocks - 1 - q % p.n_mblocks;
            } else {
                bh = q % nq;
                m_block = p.n_mblocks - 1 - q / nq;
            }
        } else if (p.persistent == 2) {
            const int nm = p.n_mblocks, npair = (nm + 1) >> 1;
            const int bid = (int)blockIdx.x;
            const int v = (bid & 7) * (g >> 3) + (bid >> 3);
            const int q = (k >> 1) * g + v;
            if (q >= nbh * npair) break;
            bh = q / npair;
            const int i = q - bh * npair;
            m_block = (k & 1) ? i : nm - 1 - i;
            if ((k & 1) && i == nm - 1 - i) continue;
        } else if (p.persistent) {
            const int lin = k * g + ((k & 1) ? g - 1 - (int)blockIdx.x : (int)blockIdx.x);
            if (lin >= nbh * p.n_mblocks) break;
            bh = lin % nbh;
            m_block = p.n_mblocks - 1 - lin / nbh;
        } else {
            if (k > 0) break;
            bh = blockIdx.x;
            m_block = gridDim.y - 1 - blockIdx.y;
        }
        fwd8w_item<F16>(p, smem, bh, m_block XFA_F8_ACC_ARG);
    }
#ifdef XFA_FWD8_STAMPS
    if ((threadIdx.x & 63) < 8) atomicAdd(&g_fwd8_stamps[(threadIdx.x >> 6) * 8 + (threadIdx.x & 63)], (unsigned long long)acc);
#endif
    if (p.persistent == 3 && threadIdx.x == 0) {
        // the grid's last workgroup resets the queue counters for the next launch on the stream
        const int total = (int)(gridDim.x * gridDim.y * gridDim.z);
        if (atomicAdd(p.work_ctr + 1, 1) == total - 1) {
            for (int i = 2; i < 10; ++i) atomicExch(p.work_ctr + i, 0);
            atomicExch(p.work_ctr + 1, 0);
        }
    }
}

}  // namespace xfa

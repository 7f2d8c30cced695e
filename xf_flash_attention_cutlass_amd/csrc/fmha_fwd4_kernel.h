// fmha_fwd4_kernel.h — 4-wave forward for D = 128 (one wave per SIMD, 64 query rows per wave).
//
// Replaces the reference's `compute_attn_1rowblock_splitkv` (flash_fwd_kernel_hip.h:585-1283)
// for the shapes the BASELINE configurations run (dense and varlen, D = 128, bf16 / fp16,
// causal / right window / none, one split): same math as fmha_fwd_kernel.h, re-structured so one
// wave owns 64 query rows (two 32-row MFMA blocks) and the whole 512-register file:
//
//  * every K fragment and every V^T fragment read from LDS feeds two MFMAs (the two row blocks),
//    half the LDS reads per MFMA of the 8-wave kernel;
//  * the key-tile loop is a three-stage pipeline — step j runs QK^T of tile j+2, the softmax of
//    tile j+1 and PV of tile j on one instruction stream — with every instruction placed in an
//    MFMA gap by tools/gen_fwd4.py;
//  * no row max in the loop: P = exp2(S c - m) against the first tile's true row max; a tile
//    whose partial row sums pass 2^fwd_slack re-runs its softmax against the true running max
//    after rescaling O and l (rare; same result up to rounding);
//  * K / V tiles arrive by LDS-DMA into 4-slot K and V rings: step j issues K_{j+4} and V_{j+2}
//    and publishes K_{j+3}, V_{j+1} at its mid-point barrier (one barrier per tile).
//
// The item's whole pipeline is one generated asm statement with a fixed register map
// (fmha_fwd4_body.h); this file computes its geometry (SRDs, per-lane offsets, tile counts).
#pragma once

#include "fmha_common.h"
#ifdef XFA_FWD4_BODY
#include XFA_FWD4_BODY          // an A/B variant of the generated body (tools/fwd4_variants.sh)
#else
#include "fmha_fwd4_body.h"
#endif

namespace xfa {

constexpr int kFwd4Rows = 256;            // query rows per workgroup (4 waves x 64)
constexpr int kFwd4Tile = 128 * 64 * 2;   // bytes of one K (or V) tile at D = 128
constexpr int kFwd4VReg = 4 * kFwd4Tile;  // V ring after the 4 K slots
constexpr int kFwd4Smem = 8 * kFwd4Tile;  // 128 KiB

__device__ __forceinline__ i32x4 fwd4_srd(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
    r[3] = 0x00020000;
    return r;
}

// One (batch x kv head, 256-row query block) item.
template <bool BF16>
__device__ __forceinline__ void fwd4_item(const FwdParams& p, char* smem, const int bh, const int m_block) {
    constexpr int HD = 128;
    // item-local copies made opaque: otherwise hipcc hoists lane- and parameter-derived values
    // out of the persistent item loop and keeps them live across the asm body
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int lr = lane & 31;
    const int hh = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int bidx = bh / p.hk;
    const int hk_i = bh - bidx * p.hk;
    int q_off = 0, sq = p.seqlen_q, k_off = 0, sk = p.seqlen_k;
    if (p.cu_seqlens_q) { q_off = p.cu_seqlens_q[bidx]; sq = p.cu_seqlens_q[bidx + 1] - q_off; }
    if (p.cu_seqlens_k) { k_off = p.cu_seqlens_k[bidx]; sk = p.cu_seqlens_k[bidx + 1] - k_off; }
    if (p.seqused_k) sk = p.seqused_k[bidx];
    const int G = p.group;
    const int rows_total = sq * G;
    const int row0 = m_block * kFwd4Rows;
    if (row0 >= rows_total) return;    // workgroup-uniform
    const int diag = sk - sq;
    auto lim_r = [&](int pos) { return p.wr >= 0 ? min(sk, pos + diag + p.wr + 1) : sk; };

    // key tiles of the workgroup: [0, ntl)
    const int pos_hi = (min(row0 + kFwd4Rows, rows_total) - 1) / G;
    const int n_hi = sk > 0 ? lim_r(pos_hi) : 0;
    const int ntl = n_hi > 0 ? (n_hi + kBlockN - 1) / kBlockN : 0;

    // this wave: rows wrow0 .. wrow0 + 63; last tile t_w; tiles >= e_w need the edge mask
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

    // per lane: the rows of the two 32-row blocks
    int qoff[2], ooff[2], loff[2], lim[2];
    const int q_row = (int)p.q_row, q_head = (int)p.q_head;
    const int o_row = (int)p.o_row, o_head = (int)p.o_head;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
        const int row = wrow0 + 32 * rb + lr;
        const bool ok = row < rows_total;
        const int pos = ok ? row / G : 0;
        const int head = hk_i * G + (ok ? row - pos * G : 0);
        qoff[rb] = ok ? (pos * q_row + head * q_head) * 2 + 16 * hh : kOOB;
        ooff[rb] = ok ? (pos * o_row + head * o_head) * 2 + 16 * hh : kOOB;
        loff[rb] = (ok && hh == 0) ? (int)(head * p.lse_head + pos) * 4 : kOOB;
        // key limit of tile 0 for this lane's keys (offset 4*hh folded in); other rows: none
        lim[rb] = (ok ? lim_r(pos) : sk) - 4 * hh;
    }

    if (ntl <= 0) {
        // no visible key for any row: O = 0, LSE = +inf (the reference's empty-row output)
        typedef __attribute__((ext_vector_type(4))) unsigned u4;
        char* oseq = reinterpret_cast<char*>(p.o) + ((int64_t)bidx * p.o_batch + (int64_t)q_off * p.o_row) * 2;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            if (ooff[rb] == kOOB) continue;
#pragma unroll
            for (int c = 0; c < 8; ++c) *reinterpret_cast<u4*>(oseq + ooff[rb] + 32 * c) = u4{0, 0, 0, 0};
            if (p.lse && hh == 0) p.lse[(int64_t)bidx * p.lse_batch + q_off + loff[rb] / 4] = INFINITY;
        }
        return;
    }

    // SRDs: Q / O / LSE of this sequence; K / V of this sequence and kv head, their range ending
    // at the workgroup's last key tile (the ring's DMA past it reads zeros and moves no bytes)
    const char* qseq = reinterpret_cast<const char*>(p.q) + ((int64_t)bidx * p.q_batch + (int64_t)q_off * p.q_row) * 2;
    char* oseq = reinterpret_cast<char*>(p.o) + ((int64_t)bidx * p.o_batch + (int64_t)q_off * p.o_row) * 2;
    const uint32_t qbytes = (uint32_t)(((int64_t)(sq - 1) * p.q_row + (int64_t)(p.h - 1) * p.q_head + HD) * 2);
    const uint32_t obytes = (uint32_t)(((int64_t)(sq - 1) * p.o_row + (int64_t)(p.h - 1) * p.o_head + HD) * 2);
    const i32x4 qsrd = fwd4_srd(qseq, qbytes), osrd = fwd4_srd(oseq, obytes);
    // LSE rows of this sequence: [h][lse_head] floats from lseq (kOOB offsets stay out of range)
    const float* lseq = p.lse ? p.lse + (int64_t)bidx * p.lse_batch + q_off : p.lse;
    const int64_t lbytes = p.lse ? ((int64_t)(p.h - 1) * p.lse_head + sq) * 4 : 0;
    const i32x4 lsrd = fwd4_srd(lseq, (uint32_t)min(lbytes, (int64_t)kOOB - 1));
    const int k_row = (int)p.k_row;
    const char* kseq = reinterpret_cast<const char*>(p.k) +
                       ((int64_t)bidx * p.k_batch + (int64_t)k_off * p.k_row + (int64_t)hk_i * p.k_head) * 2;
    const char* vseq = reinterpret_cast<const char*>(p.v) +
                       ((int64_t)bidx * p.v_batch + (int64_t)k_off * p.v_row + (int64_t)hk_i * p.v_head) * 2;
    const int nk = min(sk, ntl * kBlockN);
    const uint32_t kvbytes = (uint32_t)(((nk - 1) * k_row + HD) * 2);
    const int kblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)kseq);
    const int kbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)kseq >> 32) & 0xFFFF);
    const int vblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)vseq);
    const int vbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)vseq >> 32) & 0xFFFF);

    // per-lane DMA offsets: piece g = wave*4 + i is 8 rows x 8 chunks of the kv_off image (lane
    // l lands at g KiB + 16 l); pieces 2h and 2h+1 differ by 8 chunks (128 bytes); K and V share
    // them (k_row == v_row, checked on the host)
    int dma[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int g = wave * 4 + 2 * h;
        const int r = 8 * (g / 2) + (lane & 31) / 4;
        const int cch = 4 * (lane >> 5) + ((lane & 3) ^ ((r >> 2) & 3));
        dma[h] = r * k_row * 2 + cch * 16;
    }
    // LDS read bases (kv_off image, slot 0; the ring slots are immediate offsets)
    const int sbase = (int)(size_t)smem;
    int kb[2], vb[2];
    {
        const int q4 = (lane & 15) >> 2;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            kb[u] = sbase + kv_off<HD>(lr, 2 * u + hh);
            const int r = 8 * u + 4 * hh + q4;
            const int col = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            vb[u] = sbase + kFwd4VReg + kv_off<HD>(r, col >> 3) + 8 * ((col >> 2) & 1);
        }
    }
    const int kstep = __builtin_amdgcn_readfirstlane(kBlockN * k_row * 2);
    (void)kvbytes;
    const int kdst = __builtin_amdgcn_readfirstlane(sbase + wave * 4096);
    const float thr = __builtin_amdgcn_exp2f(p.max_slack);
    if constexpr (BF16)
        fwd4_item_bf16(kblo, kbhi, vblo, vbhi, (int)kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w,
                       p.scale_log2, thr, kb[0], kb[1], vb[0], vb[1], dma[0], dma[0] + 128, dma[1],
                       dma[1] + 128, lim[0], lim[1], qoff[0], qoff[1], ooff[0], ooff[1], loff[0], loff[1]);
    else
        fwd4_item_f16(kblo, kbhi, vblo, vbhi, (int)kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w,
                      p.scale_log2, thr, kb[0], kb[1], vb[0], vb[1], dma[0], dma[0] + 128, dma[1],
                      dma[1] + 128, lim[0], lim[1], qoff[0], qoff[1], ooff[0], ooff[1], loff[0], loff[1]);
}

// Persistent grid (one workgroup per CU) walking (b x kv head, row block) items in the
// 8-wave kernel's orders: XCD-grouped pairs (dense) or per-XCD dynamic queues (varlen).
template <bool BF16>
__global__ void __launch_bounds__(256, 1) fmha_fwd4_kernel(const FwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int s_claim[2];
    const int nbh = p.b * p.hk;
    const int g = gridDim.x;
    // static schedules: item k of this workgroup (-1: past the end, -2: a skipped index)
    auto static_item = [&](const int k, int& bh, int& m_block) -> int {
        if (p.persistent == 2) {
            const int nm = p.n_mblocks, npair = (nm + 1) >> 1;
            const int bid = (int)blockIdx.x;
            const int v = (bid & 7) * (g >> 3) + (bid >> 3);
            const int q = (k >> 1) * g + v;
            if (q >= nbh * npair) return -1;
            bh = q / npair;
            const int i = q - bh * npair;
            m_block = (k & 1) ? i : nm - 1 - i;
            return ((k & 1) && i == nm - 1 - i) ? -2 : 0;
        }
        const int lin = k * g + ((k & 1) ? g - 1 - (int)blockIdx.x : (int)blockIdx.x);
        if (lin >= nbh * p.n_mblocks) return -1;
        bh = lin % nbh;
        m_block = p.n_mblocks - 1 - lin / nbh;
        return 0;
    };
    for (int k = 0;; ++k) {
        int bh, m_block;
        if (p.persistent == 1 || p.persistent == 2) {
            const int r = static_item(k, bh, m_block);
            if (r == -1) break;
            if (r == -2) continue;
            fwd4_item<BF16>(p, smem, bh, m_block);
            continue;
        }
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
        } else {
            if (k > 0) break;
            bh = blockIdx.x;
            m_block = gridDim.y - 1 - blockIdx.y;
        }
        fwd4_item<BF16>(p, smem, bh, m_block);
    }
    if (p.persistent == 3 && threadIdx.x == 0) {
        const int total = (int)(gridDim.x * gridDim.y * gridDim.z);
        if (atomicAdd(p.work_ctr + 1, 1) == total - 1) {
            for (int i = 2; i < 10; ++i) atomicExch(p.work_ctr + i, 0);
            atomicExch(p.work_ctr + 1, 0);
        }
    }
}

}  // namespace xfa

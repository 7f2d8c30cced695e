// fmha_fwdpp_kernel.h — 8-wave "ping-pong" forward for D = 128 (two waves per SIMD, 32 query
// rows per wave).
//
// Replaces the reference's `compute_attn_1rowblock_splitkv` (flash_fwd_kernel_hip.h:585-1283)
// for the shapes the 4-wave kernel (fmha_fwd4_kernel.h) runs — dense and varlen, D = 128, bf16 /
// fp16, causal / right window / none, one split — with the same math and item (256 query rows
// of one (batch x kv head)), re-structured for two waves per SIMD:
//
//  * wave w owns rows 32w .. 32w + 31 of the item; waves w and w + 4 share a SIMD;
//  * a wave alternates an MFMA phase (PV of tile j, QK^T of tile j+1) and a VALU phase (softmax
//    of tile j+1, its share of the LDS-DMA of tile j+3), each closed by a barrier, and waves 4-7
//    run one phase behind waves 0-3: on every SIMD one wave issues MFMAs while the other issues
//    VALU / DMA (tools/gen_fwdpp.py generates the item body, fmha_fwdpp_body.h);
//  * no row max in the loop (P against tile 0's max, a rare redo past 2^fwd_slack), as the
//    4-wave kernel.
// This file computes the item geometry (SRDs, per-lane offsets, the wave's last / first-masked
// tiles) and runs the persistent item schedules of fmha_fwd4_kernel.h.
#pragma once

#include "fmha_common.h"
#ifdef XFA_FWDPP_BODY
#include XFA_FWDPP_BODY         // an A/B variant of the generated body (tools/fwdpp_variants.sh)
#else
#include "fmha_fwdpp_body.h"
#endif
#ifdef XFA_FWDPP16_BODY
#include XFA_FWDPP16_BODY
#else
#include "fmha_fwdpp16_body.h"  // the same schedule on v_mfma_f32_16x16x32 (tools/gen_fwdpp16.py)
#endif

namespace xfa {

constexpr int kFwdppRows = 256;            // query rows per workgroup (8 waves x 32)

#ifdef XFA_FWDPP_STAMPS
// Diagnostic build only (tools/fwdpp_variants.sh "name=--stamps", tools/pp_stamps.py): each wave
// sums the s_memtime cycles of every phase class (gen_fwdpp.ST_*) over its items in lanes 0-7 of
// one register; the kernel adds them into this array at its end (read by fmha_fwdpp_stamps).
static __device__ unsigned g_fwdpp_stamps[8 * 8];
#define XFA_PP_ACC_PARAM , unsigned& acc
#define XFA_PP_ACC_ARG , acc
#else
#define XFA_PP_ACC_PARAM
#define XFA_PP_ACC_ARG
#endif
constexpr int kFwdppTile = 128 * 64 * 2;   // bytes of one K (or V) tile at D = 128
constexpr int kFwdppVReg = kFwdppRing * kFwdppTile;      // the V ring follows the K ring
constexpr int kFwdppSmem = 2 * kFwdppRing * kFwdppTile;  // (kFwdppRing: the generated body's)

__device__ __forceinline__ i32x4 fwdpp_srd(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
    r[3] = 0x00020000;
    return r;
}

// The 16x16x32 body's image: kv_off with the chunk XORed by ppx16(row bits 2-3) = 0, 2, 3, 1
// instead of the bits themselves.  Its K row reads (16 lanes of a ds_read_b128 bank group cover
// rows {0-3, 12-15} at one chunk and rows {4-11} at the next) and its V^T reads (rows 4 g + q of
// lane group g) then land on distinct banks: 4 / 2 cycles instead of 8 / 4 (tools/fwdpp_banks.py;
// PMC r06: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.5 with the plain image)
__device__ __forceinline__ constexpr int ppx16(int x) { return (0x78 >> (2 * x)) & 3; }

// One (batch x kv head, 256-row query block) item.  M16: the body on the 16x16x32 MFMA shape
// (a lane holds rows l16 and 16 + l16 of its wave's 32; per-lane operands below).
template <bool BF16, bool M16, bool PG>
__device__ __forceinline__ void fwdpp_item(const FwdParams& p, char* smem, const int bh, const int m_block XFA_PP_ACC_PARAM) {
    constexpr int HD = 128;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));       // item-local: not hoisted out of the persistent loop
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
    const int row0 = m_block * kFwdppRows;
    if (row0 >= rows_total) return;    // workgroup-uniform
    const int diag = sk - sq;
    auto lim_r = [&](int pos) { return p.wr >= 0 ? min(sk, pos + diag + p.wr + 1) : sk; };

    // left window (wl >= 0, the 32x32 body only): keys [lim_l(pos), lim_r(pos))
    auto lim_l = [&](int pos) { return p.wl >= 0 ? max(0, pos + diag - p.wl) : 0; };

    // key tiles of the workgroup: [T0, T0 + ntl) — T0 > 0 when the item's first row's window
    // starts past key 0; the body counts tiles from T0 (K / V bases, limits shifted by 64 T0)
    const int pos_hi = (min(row0 + kFwdppRows, rows_total) - 1) / G;
    const int n_hi = sk > 0 ? lim_r(pos_hi) : 0;
    const int ntl_abs = n_hi > 0 ? (n_hi + kBlockN - 1) / kBlockN : 0;
    const int T0 = (M16 || ntl_abs <= 0) ? 0 : min(lim_l(row0 / G) / kBlockN, ntl_abs - 1);
    const int ntl = ntl_abs - T0;

    // this wave: rows wrow0 .. wrow0 + 31; last tile t_w; tiles >= e_w need the right edge mask,
    // tiles < l_w the left one
    const int wrow0 = row0 + 32 * wave;
    int t_w = -1, e_w = 1 << 30, l_w = 0, f_w = 0;
    if (wrow0 < rows_total && ntl > 0) {
        const int wp_lo = wrow0 / G, wp_hi = (min(wrow0 + 32, rows_total) - 1) / G;
        const int lr_hi = lim_r(wp_hi), lr_lo = lim_r(wp_lo);
        t_w = lr_hi > 0 ? min(ntl_abs, (lr_hi + kBlockN - 1) / kBlockN) - 1 - T0 : -1;
        t_w = max(t_w, -1);
        e_w = (lr_lo > 0 ? lr_lo / kBlockN : 0) - T0;
        l_w = (lim_l(wp_hi) + kBlockN - 1) / kBlockN - T0;
        f_w = lim_l(wp_lo) / kBlockN - T0;     // tiles before it: no row of the wave sees a key
    }
    t_w = __builtin_amdgcn_readfirstlane(t_w);
    e_w = __builtin_amdgcn_readfirstlane(e_w);
    l_w = __builtin_amdgcn_readfirstlane(l_w);
    f_w = __builtin_amdgcn_readfirstlane(f_w);

    // this lane's row
    const int row = wrow0 + lr;
    const bool ok = row < rows_total;
    const int pos = ok ? row / G : 0;
    const int head = hk_i * G + (ok ? row - pos * G : 0);
    const int qoff = ok ? (pos * (int)p.q_row + head * (int)p.q_head) * 2 + 16 * hh : kOOB;
    const int ooff = ok ? (pos * (int)p.o_row + head * (int)p.o_head) * 2 + 16 * hh : kOOB;
    const int loff = (ok && hh == 0) ? (int)(head * p.lse_head + pos) * 4 : kOOB;
    // key limits of tile 0 (absolute tile T0) for this lane's keys (offset 4*hh folded in);
    // other rows: none
    const int lim = (ok ? lim_r(pos) : sk) - 4 * hh - kBlockN * T0;
    const int liml = (ok ? lim_l(pos) : 0) - 4 * hh - kBlockN * T0;
    const int wid = max(lim - liml, 0);

    if (ntl <= 0) {
        // no visible key for any row: O = 0, LSE = +inf (the reference's empty-row output)
        typedef __attribute__((ext_vector_type(4))) unsigned u4;
        char* oseq = reinterpret_cast<char*>(p.o) + ((int64_t)bidx * p.o_batch + (int64_t)q_off * p.o_row) * 2;
        if (ooff != kOOB) {
#pragma unroll
            for (int c = 0; c < 8; ++c) *reinterpret_cast<u4*>(oseq + ooff + 32 * c) = u4{0, 0, 0, 0};
            if (p.lse && hh == 0) p.lse[(int64_t)bidx * p.lse_batch + q_off + loff / 4] = INFINITY;
        }
        return;
    }

    // SRDs: Q / O / LSE of this sequence; K / V of this sequence and kv head, their range ending
    // at the workgroup's last key tile (the ring's DMA past it reads zeros and moves no bytes)
    const char* qseq = reinterpret_cast<const char*>(p.q) + ((int64_t)bidx * p.q_batch + (int64_t)q_off * p.q_row) * 2;
    char* oseq = reinterpret_cast<char*>(p.o) + ((int64_t)bidx * p.o_batch + (int64_t)q_off * p.o_row) * 2;
    const uint32_t qbytes = (uint32_t)(((int64_t)(sq - 1) * p.q_row + (int64_t)(p.h - 1) * p.q_head + HD) * 2);
    const uint32_t obytes = (uint32_t)(((int64_t)(sq - 1) * p.o_row + (int64_t)(p.h - 1) * p.o_head + HD) * 2);
    const i32x4 qsrd = fwdpp_srd(qseq, qbytes), osrd = fwdpp_srd(oseq, obytes);
    const float* lseq = p.lse ? p.lse + (int64_t)bidx * p.lse_batch + q_off : p.lse;
    const int64_t lbytes = p.lse ? ((int64_t)(p.h - 1) * p.lse_head + sq) * 4 : 0;
    const i32x4 lsrd = fwdpp_srd(lseq, (uint32_t)min(lbytes, (int64_t)kOOB - 1));
    const int k_row = (int)p.k_row;
    const int64_t k0 = (int64_t)k_off + (int64_t)kBlockN * T0;   // the item's first key row
    const char* kseq = reinterpret_cast<const char*>(p.k) +
                       ((int64_t)bidx * p.k_batch + k0 * p.k_row + (int64_t)hk_i * p.k_head) * 2;
    const char* vseq = reinterpret_cast<const char*>(p.v) +
                       ((int64_t)bidx * p.v_batch + k0 * p.v_row + (int64_t)hk_i * p.v_head) * 2;
    const int nk = min(sk, ntl_abs * kBlockN) - kBlockN * T0;
    const int kvbytes = __builtin_amdgcn_readfirstlane((int)(((nk - 1) * k_row + HD) * 2));
    const int kblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)kseq);
    const int kbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)kseq >> 32) & 0xFFFF);
    const int vblo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)vseq);
    const int vbhi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)vseq >> 32) & 0xFFFF);

    // LDS-DMA: wave w loads 8-row block w of every K / V tile, pieces i = chunks 8i .. 8i+7 of
    // the kv_off image (lane l lands at +16 l); K and V share the offsets (k_row == v_row)
    // (M16: the chunk XOR by row bits 2-3 goes through ppx16, so the 16x16x32 body's K row and
    // V^T reads are conflict-free too; see ppx16)
    // (paged: the descriptor base points at the wave's 8 rows, so the row offset is lr / 4)
    const int r = 8 * wave + lr / 4;
    const int cch = 4 * hh + ((lane & 3) ^ (M16 ? ppx16((r >> 2) & 3) : ((r >> 2) & 3)));
    const int dma0 = (PG ? lr / 4 : r) * k_row * 2 + cch * 16;
    // LDS read bases (kv_off image, slot 0; the ring slots are immediate offsets)
    const int sbase = (int)(size_t)smem;
    int kb[2], vb[2];
    {
        const int q4 = (lane & 15) >> 2;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            kb[u] = sbase + kv_off<HD>(lr, 2 * u + hh);
            const int rr = 8 * u + 4 * hh + q4;
            const int col = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            vb[u] = sbase + kFwdppVReg + kv_off<HD>(rr, col >> 3) + 8 * ((col >> 2) & 1);
        }
    }
    const int kstep = __builtin_amdgcn_readfirstlane(kBlockN * k_row * 2);
    const int kdst = __builtin_amdgcn_readfirstlane(sbase + wave * 2048);
    const int grp = __builtin_amdgcn_readfirstlane(wave >> 2);
    const float thr = __builtin_amdgcn_exp2f(p.max_slack);
    if constexpr (M16) {
        static_assert(kFwdpp16Ring == kFwdppRing, "both bodies address the same LDS ring");
        // row tile rt of this lane: row wrow0 + 16 rt + l16, 4 keys per 16-key block from 4 g
        const int g = lane >> 4, l16 = lane & 15;
        int qo[2], oo[2], lo[2], li[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int rrow = wrow0 + 16 * rt + l16;
            const bool rok = rrow < rows_total;
            const int rpos = rok ? rrow / G : 0;
            const int rhead = hk_i * G + (rok ? rrow - rpos * G : 0);
            qo[rt] = rok ? (rpos * (int)p.q_row + rhead * (int)p.q_head) * 2 + 16 * g : kOOB;  // chunk 4 s + g
            oo[rt] = rok ? (rpos * (int)p.o_row + rhead * (int)p.o_head) * 2 + 8 * g : kOOB;   // d 16 dt + 4 g
            lo[rt] = (rok && g == 0) ? (int)(rhead * p.lse_head + rpos) * 4 : kOOB;
            li[rt] = (rok ? lim_r(rpos) : sk) - 4 * g;
        }
        // K row reads: key 16 kt + l16, chunk 4 s + g; V^T reads: lane 4 q + p of group g, key
        // 4 g + q (+ 32 ks + 16 h), d 16 dt + 4 p, base per dt parity e (kv_off image)
        const int kb0 = sbase + 2048 * ((lane >> 3) & 1) + 64 * (lane & 7) + 16 * (g ^ ppx16((lane >> 2) & 3));
        const int q4 = (lane & 15) >> 2, p4 = lane & 3;
        int vb16[2];
#pragma unroll
        for (int e = 0; e < 2; ++e)
            vb16[e] = sbase + kFwdppVReg + 2048 * (g >> 1) + 64 * (4 * (g & 1) + q4) +
                      16 * ((2 * e + (p4 >> 1)) ^ ppx16(g)) + 8 * (p4 & 1);
#ifdef XFA_FWDPP16_STAMPS
#define XFA_PP16_ACC_ARG , acc
#else
#define XFA_PP16_ACC_ARG
#endif
        if constexpr (BF16)
            fwdpp16_item_bf16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w, grp,
                              p.scale_log2, thr, kb0, vb16[0], vb16[1], dma0, dma0 + 128, li[0], li[1], qo[0], qo[1],
                              oo[0], oo[1], lo[0], lo[1] XFA_PP16_ACC_ARG);
        else
            fwdpp16_item_f16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w, grp,
                             p.scale_log2, thr, kb0, vb16[0], vb16[1], dma0, dma0 + 128, li[0], li[1], qo[0], qo[1],
                             oo[0], oo[1], lo[0], lo[1] XFA_PP16_ACC_ARG);
#undef XFA_PP16_ACC_ARG
        return;
    }
    // score features (gen_fwdpp.feature_block): bit 0 softcap, bit 1 ALiBi (the lane's row slope
    // in raw-score units and its distance pos + diag - 4 hh to the lane's key offset 0)
    // bit 2: causal ALiBi (wr = 0, every visible key <= pos + diag) in the linear frame +w key
    // (gen_fwdpp._alibi_linear_ops: one v_fmac per score instead of the |.| form's two)
    const bool lin = p.alibi && p.wr == 0;
    const int feat = __builtin_amdgcn_readfirstlane((p.softcap_pre > 0.f ? 1 : 0) | (p.alibi ? (lin ? 4 : 2) : 0));
    const float scp2 = p.softcap_pre * (2.f * kLog2e);
    const float alw = (p.alibi && ok) ? p.alibi[bidx * p.alibi_bstride + head] * p.alibi_mul : 0.f;
    // |.| form: the distance base pos + diag - 4 hh - 64 T0; linear form: c w (64 T0 + 4 hh), the
    // tile-invariant part of the frame shift c w key0
    const float ald = lin ? p.scale_log2 * alw * (float)(kBlockN * T0 + 4 * hh)
                          : (float)(pos + diag - 4 * hh - kBlockN * T0);
    const float alw2 = p.scale_log2 * alw;                       // c w
    const float adiag = p.scale_log2 * alw * (float)(pos + diag);   // the |.| form's row offset
    // the row's best ALiBi bias: -w times the distance from pos + diag to its nearest visible key
    // (keys [lim_l, lim_r)); tile 0's reference max is lifted by it
    const int hi_k = ok ? lim_r(pos) : 0, lo_k = ok ? lim_l(pos) : 0;
    const int near = min(max(pos + diag, lo_k), max(hi_k - 1, lo_k));
    const float alm = hi_k > lo_k ? (lin ? alw * (float)near : -alw * (float)abs(pos + diag - near)) : 0.f;
    if constexpr (PG) {
#ifndef XFA_FWDPP_STAMPS
        // paged K/V (gen_fwdpp.py PAGED): per tile, each wave's 8 rows sit in one page (page size
        // a power of two >= 8, fwd4_eligible); the body loads the page id from this sequence's
        // block-table row and builds the wave's descriptors from the pools' bases (kblo.. here:
        // pool + this kv head's offset), the page stride and the row bytes
        const int* btab = p.block_table + (int64_t)bidx * p.bt_stride;
        const char* kpool = reinterpret_cast<const char*>(p.k) + (int64_t)hk_i * p.k_head * 2;
        const char* vpool = reinterpret_cast<const char*>(p.v) + (int64_t)hk_i * p.v_head * 2;
        const int pkl = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)kpool);
        const int pkh = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)kpool >> 32) & 0xFFFF);
        const int pvl = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)vpool);
        const int pvh = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)vpool >> 32) & 0xFFFF);
        const int pstr = __builtin_amdgcn_readfirstlane((int)(p.k_batch * 2));
        const int rowb = __builtin_amdgcn_readfirstlane(k_row * 2);
        const int lgp = __builtin_amdgcn_readfirstlane(31 - __builtin_clz(p.page_size));
        const int pmask = __builtin_amdgcn_readfirstlane(p.page_size - 1);
        const int skv = __builtin_amdgcn_readfirstlane(sk);
        const int skey0 = __builtin_amdgcn_readfirstlane(kBlockN * T0 + 8 * wave);
        if constexpr (BF16)
            fwdpp_pg_item_bf16(pkl, pkh, pvl, pvh, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w, grp,
                               p.scale_log2, thr, kb[0], kb[1], vb[0], vb[1], dma0, dma0 + 128, lim, qoff, ooff,
                               loff, feat, scp2, alw, ald, alm, l_w, liml, wid, f_w, alw2, adiag, btab, pstr, rowb,
                               lgp, pmask, skv, skey0);
        else
            fwdpp_pg_item_f16(pkl, pkh, pvl, pvh, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w, grp,
                              p.scale_log2, thr, kb[0], kb[1], vb[0], vb[1], dma0, dma0 + 128, lim, qoff, ooff,
                              loff, feat, scp2, alw, ald, alm, l_w, liml, wid, f_w, alw2, adiag, btab, pstr, rowb,
                              lgp, pmask, skv, skey0);
#endif
        return;
    }
    if constexpr (BF16)
        fwdpp_item_bf16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w, grp,
                        p.scale_log2, thr, kb[0], kb[1], vb[0], vb[1], dma0, dma0 + 128, lim, qoff, ooff, loff,
                        feat, scp2, alw, ald, alm, l_w, liml, wid, f_w, alw2, adiag XFA_PP_ACC_ARG);
    else
        fwdpp_item_f16(kblo, kbhi, vblo, vbhi, kvbytes, qsrd, osrd, lsrd, kstep, kdst, ntl, t_w, e_w, grp,
                       p.scale_log2, thr, kb[0], kb[1], vb[0], vb[1], dma0, dma0 + 128, lim, qoff, ooff, loff,
                       feat, scp2, alw, ald, alm, l_w, liml, wid, f_w, alw2, adiag XFA_PP_ACC_ARG);
}

// Persistent grid (one workgroup per CU) over the items, the 4-wave kernel's orders: XCD-grouped
// (n-1-i, i) row-block pairs (dense) or per-XCD dynamic queues (varlen).
template <bool BF16, bool M16 = false, bool PG = false>
__global__ void __launch_bounds__(512, 1) fmha_fwdpp_kernel(const FwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int s_claim[2];
    const int nbh = p.b * p.hk;
    const int g = gridDim.x;
#ifdef XFA_FWDPP_STAMPS
    unsigned acc = 0;
#endif
    for (int k = 0;; ++k) {
        int bh, m_block;
        if (p.persistent == 2) {
            const int nm = p.n_mblocks, npair = (nm + 1) >> 1;
            const int bid = (int)blockIdx.x;
            const int v = (bid & 7) * (g >> 3) + (bid >> 3);
            const int q = (k >> 1) * g + v;
            if (q >= nbh * npair) break;
            bh = q / npair;
            const int i = q - bh * npair;
            m_block = (k & 1) ? i : nm - 1 - i;
            if ((k & 1) && i == nm - 1 - i) continue;
        } else if (p.persistent == 1) {
            const int lin = k * g + ((k & 1) ? g - 1 - (int)blockIdx.x : (int)blockIdx.x);
            if (lin >= nbh * p.n_mblocks) break;
            bh = lin % nbh;
            m_block = p.n_mblocks - 1 - lin / nbh;
        } else if (p.persistent == 3) {
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
        fwdpp_item<BF16, M16, PG>(p, smem, bh, m_block XFA_PP_ACC_ARG);
    }
#ifdef XFA_FWDPP_STAMPS
    if ((threadIdx.x & 63) < 8) atomicAdd(&g_fwdpp_stamps[(threadIdx.x >> 6) * 8 + (threadIdx.x & 63)], acc);
#endif
    if (p.persistent == 3 && threadIdx.x == 0) {
        const int total = (int)(gridDim.x * gridDim.y * gridDim.z);
        if (atomicAdd(p.work_ctr + 1, 1) == total - 1) {
            for (int i = 2; i < 10; ++i) atomicExch(p.work_ctr + i, 0);
            atomicExch(p.work_ctr + 1, 0);
        }
    }
}

}  // namespace xfa

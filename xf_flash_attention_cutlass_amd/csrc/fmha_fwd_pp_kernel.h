// fmha_fwd_pp_kernel.h — ping-pong forward for gfx950: same math and operand layouts as
// fmha_fwd_kernel.h, different schedule.
//
// 8 waves = 2 groups of 4; waves w and w+4 share a SIMD (MI355X_MICROARCH.md §Two waves per
// SIMD).  Each K/V tile takes two barrier-separated slots.  In every slot one group runs its
// MFMA segment  [O^T += V(j-1)^T P(j-1)^T ; S^T(j) = K(j) Q^T]  while its SIMD partner runs its
// VALU segment  [mask, online softmax of S(j'), O rescale, P -> bf16], so each SIMD pairs a
// matrix stream with a vector stream instead of two copies of the same phase:
//
//   slot 2u+1: group 0 MSEG(u)       group 1 VSEG(u-1)
//   slot 2u+2: group 0 VSEG(u)       group 1 MSEG(u)
//
// Tile staging: each wave issues its share of the global loads of K(u+1) and V(u) before
// VSEG(u-1) and writes them to LDS after MSEG(u) (two slots of latency cover), into
// double-buffered K and V images (see the loop for the hazard argument).  Q is staged in LDS
// once (the VGPR budget at 2 waves/SIMD holds O, S, P and the staging registers).
#pragma once

#include "fmha_common.h"

namespace xfa {

template <int HD, typename T, bool MASK, bool FEAT, int SCHED = 0>
__global__ void __launch_bounds__(512, 2) fmha_fwd_pp_kernel(const FwdParams p) {
    using V8 = typename DT<T>::v8;
    constexpr int NW = 8;
    constexpr int NT = NW * 64;
    constexpr int BM = NW * 32;
    constexpr int CPR = HD / 8;
    constexpr int NLD = kBlockN * CPR / NT;
    constexpr int TILE = kBlockN * HD * 2;
    constexpr int NS = HD / 16;
    constexpr int ND = HD / 32;
    static_assert(NLD >= 1 && (NT % CPR) == 0, "tile/thread geometry");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* kbuf = smem;                 // [2][TILE]
    char* vbuf = smem + 2 * TILE;      // [2][TILE]
    char* qbuf = smem + 4 * TILE;      // [BM][HD] (Q stays in LDS: VGPR budget at 2 waves/SIMD)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int lr = lane & 31;
    const int hh = lane >> 5;
    const bool mfirst = __builtin_amdgcn_readfirstlane(wave) < NW / 2;

    const int bh = blockIdx.x;
    const int bidx = bh / p.hk;
    const int hk_i = bh - bidx * p.hk;
    const int m_block = gridDim.y - 1 - blockIdx.y;
    const int split = blockIdx.z;

    int q_off = 0, sq = p.seqlen_q, k_off = 0, sk = p.seqlen_k;
    if (p.cu_seqlens_q) { q_off = p.cu_seqlens_q[bidx]; sq = p.cu_seqlens_q[bidx + 1] - q_off; }
    if (p.cu_seqlens_k) { k_off = p.cu_seqlens_k[bidx]; sk = p.cu_seqlens_k[bidx + 1] - k_off; }
    if (p.seqused_k) sk = p.seqused_k[bidx];
    const int G = p.group;
    const int rows_total = sq * G;
    const int row0 = m_block * BM;
    if (row0 >= rows_total) return;

    const int diag = sk - sq;
    auto lim_r = [&](int pos) { return (MASK && p.wr >= 0) ? min(sk, pos + diag + p.wr + 1) : sk; };
    auto lim_l = [&](int pos) { return (MASK && p.wl >= 0) ? max(0, pos + diag - p.wl) : 0; };
    const int pos_lo = row0 / G;
    const int pos_hi = (min(row0 + BM, rows_total) - 1) / G;
    const int n_lo = lim_l(pos_lo);
    const int n_hi = lim_r(pos_hi);
    int nb_lo = n_lo / kBlockN;
    int nb_hi = n_hi > n_lo ? (n_hi + kBlockN - 1) / kBlockN : nb_lo;
    const bool is_split = p.num_splits > 1;
    if (is_split) {
        const int per = (nb_hi - nb_lo + p.num_splits - 1) / p.num_splits;
        const int s_lo = nb_lo + split * per;
        nb_hi = min(nb_hi, s_lo + per);
        nb_lo = min(s_lo, nb_hi);
    }
    const int nblk = nb_hi - nb_lo;

    const int wrow0 = row0 + wave * 32;
    const int row = wrow0 + lr;
    const bool row_ok = row < rows_total;
    const int pos = row_ok ? row / G : 0;
    const int head = hk_i * G + (row_ok ? row - pos * G : 0);
    const bool wave_ok = wrow0 < rows_total;
    const int wp_lo = wrow0 / G;
    const int wp_hi = (min(wrow0 + 32, rows_total) - 1) / G;
    const int w_lr_min = lim_r(wp_lo), w_lr_max = lim_r(wp_hi);
    const int w_ll_min = lim_l(wp_lo), w_ll_max = lim_l(wp_hi);
    const int my_lr = lim_r(pos), my_ll = lim_l(pos);

    float alibi_w = 0.f;
    if (FEAT && p.alibi) alibi_w = p.alibi[bidx * p.alibi_bstride + head] * p.alibi_mul;
    const float c = p.scale_log2;

    // ---- Q tile (BM rows of this workgroup) -> LDS, swizzled like K; row = local row index
    {
        const T* qseq = reinterpret_cast<const T*>(p.q) + (int64_t)bidx * p.q_batch + (int64_t)q_off * p.q_row;
        const uint32_t qbytes = (uint32_t)(((int64_t)(sq - 1) * p.q_row + (int64_t)(p.h - 1) * p.q_head + p.d) * 2);
        const __amdgpu_buffer_rsrc_t qr = make_rsrc(qseq, qbytes);
        for (int i = tid; i < BM * CPR; i += NT) {
            const int rr = i / CPR, cc = i % CPR;
            const int grow = row0 + rr;
            const int qpos = grow / G;
            const int qhead = hk_i * G + (grow - qpos * G);
            const bool ok = grow < rows_total && cc * 8 < p.d;
            const int off = ok ? (int)(((int64_t)qpos * p.q_row + (int64_t)qhead * p.q_head) * 2) + cc * 16 : kOOB;
            *reinterpret_cast<u32x4*>(qbuf + lds_off<HD>(rr, cc)) = buf_load16(qr, off);
        }
    }

    // ---- tile loader
    const int lc = tid % CPR;
    const int lrow0 = tid / CPR;
    constexpr int LROW_STEP = NT / CPR;
    const bool lc_ok = lc * 8 < p.d;
    const bool paged = FEAT && p.block_table != nullptr;
    const T* kseq = reinterpret_cast<const T*>(p.k) + (int64_t)bidx * p.k_batch + (int64_t)k_off * p.k_row +
                    (int64_t)hk_i * p.k_head;
    const T* vseq = reinterpret_cast<const T*>(p.v) + (int64_t)bidx * p.v_batch + (int64_t)k_off * p.v_row +
                    (int64_t)hk_i * p.v_head;
    const __amdgpu_buffer_rsrc_t krs =
        make_rsrc(kseq, (uint32_t)(((int64_t)(sk > 0 ? sk - 1 : 0) * p.k_row + p.d) * 2));
    const __amdgpu_buffer_rsrc_t vrs =
        make_rsrc(vseq, (uint32_t)(((int64_t)(sk > 0 ? sk - 1 : 0) * p.v_row + p.d) * 2));
    const T* kpool = reinterpret_cast<const T*>(p.k) + (int64_t)hk_i * p.k_head + lc * 8;
    const T* vpool = reinterpret_cast<const T*>(p.v) + (int64_t)hk_i * p.v_head + lc * 8;
    const int* btab = paged ? p.block_table + (int64_t)bidx * p.bt_stride : nullptr;

    auto load_rows = [&](int nb, bool is_v, u32x4 (&dst)[NLD]) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int n = nb * kBlockN + lrow0 + i * LROW_STEP;
            const bool ok = lc_ok && n < sk;
            if (paged) {
                const int nc = ok ? n : 0;
                const int pi = nc / p.page_size;
                const int pg = btab[pi];
                const int pr = nc - pi * p.page_size;
                const T* src = is_v ? vpool + (int64_t)pg * p.v_batch + (int64_t)pr * p.v_row
                                    : kpool + (int64_t)pg * p.k_batch + (int64_t)pr * p.k_row;
                const u32x4 x = *reinterpret_cast<const u32x4*>(src);
                dst[i] = ok ? x : u32x4{0, 0, 0, 0};
            } else if (is_v) {
                dst[i] = buf_load16(vrs, ok ? n * (int)p.v_row * 2 + lc * 16 : kOOB);
            } else {
                dst[i] = buf_load16(krs, ok ? n * (int)p.k_row * 2 + lc * 16 : kOOB);
            }
        }
    };
    auto store_rows = [&](char* dstbuf, const u32x4 (&src)[NLD]) {
#pragma unroll
        for (int i = 0; i < NLD; ++i)
            *reinterpret_cast<u32x4*>(dstbuf + lds_off<HD>(lrow0 + i * LROW_STEP, lc)) = src[i];
    };

    int koff[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) koff[s] = lds_off<HD>(lr, 2 * s + hh);
    const int q4 = (lane & 15) >> 2;
    int voff[2][ND];
#pragma unroll
    for (int part = 0; part < 2; ++part)
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
            const int r = 4 * hh + q4 + 8 * part;
            const int col = 32 * dt + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            voff[part][dt] = lds_off<HD>(r, col >> 3) + 8 * ((col >> 2) & 1);
        }

    f32x16 acc_o[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) acc_o[dt] = f32x16{};
    float m_run = -INFINITY, l_run = 0.f;
    f32x16 st[2] = {f32x16{}, f32x16{}};
    V8 pf[4];                      // P(j) as the four 16-key B fragments of the PV product
#pragma unroll
    for (int i = 0; i < 4; ++i) pf[i] = V8{};

    auto active = [&](int j) {     // does this wave see any key of tile j (relative index)?
        const int n0 = (nb_lo + j) * kBlockN;
        return wave_ok && n0 < w_lr_max && n0 + kBlockN > w_ll_min;
    };
    // MFMA segment: O^T += V(t-1)^T P(t-1)^T ; S^T(t) = K(t) Q^T
    auto mseg = [&](int t) {
        if (t >= 1 && active(t - 1)) {
            const char* vs = vbuf + ((t - 1) & 1) * TILE;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int rbase = 16 * ks * HD * 2;
#pragma unroll
                for (int dt = 0; dt < ND; ++dt) {
                    const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vs + rbase + voff[0][dt]));
                    const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vs + rbase + voff[1][dt]));
                    const s16x8 av = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
                    acc_o[dt] = DT<T>::mfma32(__builtin_bit_cast(V8, av), pf[ks], acc_o[dt]);
                }
            }
            if constexpr (SCHED & 1) {
                // pin a read-ahead interleave: 6 tr-reads up front, then 2 per MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
                for (int i = 0; i < 13; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
            }
        }
        if (t < nblk && active(t)) {
            const char* ks_ = kbuf + (t & 1) * TILE;
            const char* qs_ = qbuf + wave * 32 * HD * 2;   // 32-row offset keeps the swizzle
            st[0] = f32x16{};
            st[1] = f32x16{};
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const V8 b = *reinterpret_cast<const V8*>(qs_ + koff[s]);
                const V8 a0 = *reinterpret_cast<const V8*>(ks_ + koff[s]);
                const V8 a1 = *reinterpret_cast<const V8*>(ks_ + 32 * HD * 2 + koff[s]);
                st[0] = DT<T>::mfma32(a0, b, st[0]);
                st[1] = DT<T>::mfma32(a1, b, st[1]);
            }
            if constexpr (SCHED & 2) {
                // 24 b128 reads for 16 MFMAs: 6 up front, then 3 per 2 MFMAs
                __builtin_amdgcn_sched_group_barrier(0x100, 6, 1);
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 1);
            }
        }
    };
    // VALU segment: mask + online softmax of S(t), O rescale, P(t) -> fragments
    auto vseg = [&](int t) {
        if (t < 0 || t >= nblk || !active(t)) return;
        const int n0 = (nb_lo + t) * kBlockN;
        if (FEAT && p.softcap_pre > 0.f) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) st[kt][r] = fast_tanh(st[kt][r] * p.softcap_pre);
        }
        const int keyb = n0 + 4 * hh;
        if (FEAT && p.alibi) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = keyb + 32 * kt + (r & 3) + 8 * (r >> 2);
                    st[kt][r] -= alibi_w * (float)abs(pos + diag - key);
                }
        }
        if ((n0 + kBlockN > w_lr_min) || (n0 < w_ll_max)) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = keyb + 32 * kt + (r & 3) + 8 * (r >> 2);
                    if (key >= my_lr || key < my_ll) st[kt][r] = -INFINITY;
                }
        }
        float mx = st[0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, st[0][r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[1][r]);
        mx = wave_max_halves(mx);
        const float m_new = fmaxf(m_run, mx);
        const float mref = (m_new == -INFINITY) ? 0.f : m_new * c;
        if (__any(m_new > m_run)) {
            const float alpha = fast_exp2(m_run * c - mref);
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < ND; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc_o[dt][r] *= alpha;
            m_run = m_new;
        }
        float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float e = fast_exp2(fmaf(st[kt][8 * sp + j], c, -mref));
                    rs[j & 3] += e;
                    pf[2 * kt + sp][j] = (T)e;
                }
        l_run += (rs[0] + rs[1]) + (rs[2] + rs[3]);
    };

    // ---- prologue: K(0) -> kbuf[0]
    u32x4 kr[NLD], vr[NLD];
    if (nblk > 0) {
        load_rows(nb_lo, false, kr);
        store_rows(kbuf, kr);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);     // retire Q + K(0) loads (see fmha_fwd_kernel.h)
    __syncthreads();

    // One code path for both groups: [issue K(u+1), V(u) loads; VSEG(u-1); barrier; MSEG(u);
    // write K(u+1), V(u) to LDS; barrier].  Group 1 lags group 0 by one slot (one extra
    // s_barrier before its loop, group 0 takes the matching one after), so in every slot
    // one group runs MSEG and its SIMD partner runs VSEG.  Hazards: K(u+1)/V(u) are written
    // into the buffers of K(u-1)/V(u-2), whose last readers (MSEG(u-1)) are >= 1 barrier
    // older, and are read by MSEG(u+1)/PV(u), >= 1 barrier after both groups wrote them.
    // Two code orders per group would double the live ranges (measured: +100 VGPRs).
    if (!mfirst) __syncthreads();
    for (int u = 0; u <= nblk && nblk > 0; ++u) {
        const bool ld_k = u + 1 < nblk, ld_v = u < nblk;
        if (ld_k) load_rows(nb_lo + u + 1, false, kr);
        if (ld_v) load_rows(nb_lo + u, true, vr);
        vseg(u - 1);
        __syncthreads();
        mseg(u);
        if (ld_k) store_rows(kbuf + ((u + 1) & 1) * TILE, kr);
        if (ld_v) store_rows(vbuf + (u & 1) * TILE, vr);
        __syncthreads();
    }
    if (mfirst && nblk > 0) __syncthreads();

    // ---- epilogue (identical to fmha_fwd_kernel.h)
    const float l_full = wave_sum_halves(l_run);
    const bool empty = (l_full == 0.f) || (l_full != l_full);
    const float inv = empty ? 1.f : 1.f / l_full;
    if (!row_ok) return;
    if (is_split) {
        const int64_t rid = (((int64_t)split * p.b + bidx) * p.h + head) * p.seqlen_q + pos;
        float* oa = p.oaccum + rid * HD;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hh;
                f32x4 v = {acc_o[dt][4 * g] * inv, acc_o[dt][4 * g + 1] * inv,
                           acc_o[dt][4 * g + 2] * inv, acc_o[dt][4 * g + 3] * inv};
                *reinterpret_cast<f32x4*>(oa + d) = v;
            }
        if (hh == 0) p.lseaccum[rid] = empty ? -INFINITY : (m_run * c + __log2f(l_full)) * kLn2;
        return;
    }
    T* orow = reinterpret_cast<T*>(p.o) + (int64_t)bidx * p.o_batch +
              (int64_t)(q_off + pos) * p.o_row + (int64_t)head * p.o_head;
    if (p.store8) store_o_row8<T, ND>(orow, acc_o, inv, p.d, hh);
    else store_o_row16<T, ND>(orow, acc_o, inv, p.d, hh);
    if (p.lse && hh == 0) {
        p.lse[(int64_t)bidx * p.lse_batch + (int64_t)head * p.lse_head + q_off + pos] =
            empty ? INFINITY : (m_run * c + __log2f(l_full)) * kLn2;
    }
}

}  // namespace xfa

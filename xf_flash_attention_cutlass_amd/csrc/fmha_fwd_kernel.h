// fmha_fwd_kernel.h — fused QK^T -> online softmax -> PV forward for gfx950 (CDNA4).
//
// Replaces the reference's hot kernel `compute_attn_1rowblock_splitkv`
// (csrc/flash_attn/src/flash_fwd_kernel_hip.h:585-1283) and its combine
// `combine_attn_seqk_parallel` (:1322-1568).  Same math (online softmax with exp2 and the
// scale folded into one FMA, bottom-right aligned causal/local windows, ALiBi, softcap,
// varlen, paged K/V, split-KV + LSE combine), re-designed for CDNA4:
//
//  * one workgroup = NW waves; each wave owns 32 query rows -> BLOCK_M = 32*NW rows;
//    GQA groups are packed into the row dimension (row = pos*G + g), so the G query heads
//    sharing a K/V head share every K/V tile (the reference swaps only for Sq == 1,
//    export.cpp:526-532);
//  * S^T = K * Q^T with v_mfma_f32_32x32x16_{bf16,f16}: the accumulator holds 16 keys of ONE
//    query row per lane (row = lane & 31), so row max / row sum are lane-local plus one
//    v_permlane32_swap; the P accumulator is then, after a pairwise cvt, directly the B operand
//    of O^T += V^T * P^T (no LDS round trip for P) and the O^T accumulator keeps one query row
//    per lane, so the online-softmax rescale is lane-local too;
//  * K and V tiles (64 keys x HD) are register-staged into a double-buffered, XOR-swizzled LDS
//    image (one barrier per tile); K is read with ds_read_b128, V with the gfx950 transposing
//    ds_read_b64_tr_b16 — both conflict-free on the same image;
//  * masking runs only on the tiles that cross a window edge; tiles a wave cannot see are
//    skipped by that wave (wave-uniform branch); the heaviest causal row blocks launch first.
#pragma once

#include "fmha_common.h"

#include <type_traits>

namespace xfa {

#ifndef XFA_SCHED_FENCE
#define XFA_SCHED_FENCE 1
#endif
constexpr bool SCHED_FENCE = XFA_SCHED_FENCE;


// One work item = (batch x kv-head, query row block, split).
template <int HD, typename T, int NW, bool MASK, bool FEAT>
__device__ __forceinline__ void fwd_item(const FwdParams& p, char* smem, const int bh,
                                         const int m_block, const int split) {
    using V8 = typename DT<T>::v8;
    constexpr int NT = NW * 64;
    constexpr int BM = NW * 32;
    constexpr int CPR = HD / 8;                 // 16-byte chunks per K/V row
    constexpr int NLD = kBlockN * CPR / NT;     // chunks per thread per tile
    constexpr int TILE = kBlockN * HD * 2;      // bytes of one K (or V) tile
    // LDS buffers (K and V tile each): D <= 128 runs the 4-buffer LDS-DMA pipeline; D = 256
    // (32 KiB tiles) only the double-buffered register-staged loop, 128 KiB of LDS
    constexpr int NBUF = fwd_nbuf(HD);
    constexpr bool PIPE = HD <= 128;
    constexpr int VREG = NBUF * TILE;           // LDS: K tiles of buffers 0..3, then V tiles
    constexpr int NS = HD / 16;                 // k-steps of the QK^T product
    constexpr int ND = HD / 32;                 // 32-wide d tiles of O^T
    static_assert(NLD >= 1 && (NT % CPR) == 0, "tile/thread geometry");

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int lr = lane & 31;
    const int hh = lane >> 5;

    const int bidx = bh / p.hk;
    const int hk_i = bh - bidx * p.hk;

    int q_off = 0, sq = p.seqlen_q, k_off = 0, sk = p.seqlen_k;
    // varlen / seqused_k: scalar offsets only (not a FEAT specialisation)
    if (p.cu_seqlens_q) { q_off = p.cu_seqlens_q[bidx]; sq = p.cu_seqlens_q[bidx + 1] - q_off; }
    if (p.cu_seqlens_k) { k_off = p.cu_seqlens_k[bidx]; sk = p.cu_seqlens_k[bidx + 1] - k_off; }
    if (p.seqused_k) sk = p.seqused_k[bidx];
    // cache_leftpad (block_info.h leftpad_k): the sequence is cache rows [lp, sk)
    const int lp = p.leftpad_k ? p.leftpad_k[bidx] : 0;
    sk -= lp;
    const int G = p.group;
    const int rows_total = sq * G;
    const int row0 = m_block * BM;
    if (row0 >= rows_total) return;

    const int diag = sk - sq;
    // Window limits for query position `pos`: keys [lim_l, lim_r).
    auto lim_r = [&](int pos) { return (MASK && p.wr >= 0) ? min(sk, pos + diag + p.wr + 1) : sk; };
    auto lim_l = [&](int pos) { return (MASK && p.wl >= 0) ? max(0, pos + diag - p.wl) : 0; };

    // Key-tile range of the whole workgroup (and of this split).
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

    // This lane's query row.
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

    // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[row][16s + 8hh .. +7]
    V8 qf[NS];
    {
        const T* qseq = reinterpret_cast<const T*>(p.q) + (int64_t)bidx * p.q_batch + (int64_t)q_off * p.q_row;
        const uint32_t qbytes = (uint32_t)(((int64_t)(sq - 1) * p.q_row + (int64_t)(p.h - 1) * p.q_head + p.d) * 2);
        const __amdgpu_buffer_rsrc_t qr = make_rsrc(qseq, qbytes);
        // column part as an immediate offset; the asm keeps per-column offsets from being
        // hoisted out of the persistent item loop (and spilled)
        int hh_q = hh;
        asm volatile("" : "+v"(hh_q));
        const int qrow_off = row_ok ? (int)(((int64_t)pos * p.q_row + (int64_t)head * p.q_head) * 2) + 16 * hh_q : kOOB;
        const bool full_d = p.d == HD;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int off = (full_d || 16 * s + 8 * hh_q < p.d) ? qrow_off : kOOB;
            qf[s] = __builtin_bit_cast(V8, buf_load16(qr, off + 32 * s));
        }
    }

    // ---- K/V tile loader (register staged: issue early, write to LDS late)
    const int lc = tid % CPR;
    const int lrow0 = tid / CPR;
    constexpr int LROW_STEP = NT / CPR;
    const bool lc_ok = lc * 8 < p.d;
    const bool paged = FEAT && p.block_table != nullptr;
    // fp8 (OCP e4m3fn) K/V: 1-byte elements, dequantised to T with the per-tensor scale while
    // staging (the LDS image and everything after it are unchanged)
    const bool kv8 = FEAT && p.kv_fp8;
    const int esz = kv8 ? 1 : 2;
    // dense / varlen: one SRD per K and V covering this sequence's rows of this kv head
    const char* kseq = reinterpret_cast<const char*>(p.k) +
                       ((int64_t)bidx * p.k_batch + (int64_t)k_off * p.k_row + (int64_t)hk_i * p.k_head) * esz;
    const char* vseq = reinterpret_cast<const char*>(p.v) +
                       ((int64_t)bidx * p.v_batch + (int64_t)k_off * p.v_row + (int64_t)hk_i * p.v_head) * esz;
    const uint32_t kbytes = (uint32_t)(((int64_t)(sk > 0 ? sk - 1 : 0) * p.k_row + p.d) * esz);
    const uint32_t vbytes = (uint32_t)(((int64_t)(sk > 0 ? sk - 1 : 0) * p.v_row + p.d) * esz);
    const __amdgpu_buffer_rsrc_t krs = make_rsrc(kseq, kbytes);
    const __amdgpu_buffer_rsrc_t vrs = make_rsrc(vseq, vbytes);
    // paged: per-row page pointers (clamped, unconditional loads + data select)
    const char* kpool = reinterpret_cast<const char*>(p.k) + ((int64_t)hk_i * p.k_head + lc * 8) * esz;
    const char* vpool = reinterpret_cast<const char*>(p.v) + ((int64_t)hk_i * p.v_head + lc * 8) * esz;
    const int* btab = paged ? p.block_table + (int64_t)bidx * p.bt_stride : nullptr;

    u32x4 kr[NLD], vr[NLD];
    auto load_to = [&](int nb, u32x4 (&ko)[NLD], u32x4 (&vo)[NLD]) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int n = nb * kBlockN + lrow0 + i * LROW_STEP;
            const bool ok = lc_ok && n < sk;
            if (paged) {
                const int nc = (ok ? n : 0) + lp;
                const int pi = nc / p.page_size;
                const int pg = btab[pi];
                const int pr = nc - pi * p.page_size;
                const char* ka = kpool + ((int64_t)pg * p.k_batch + (int64_t)pr * p.k_row) * esz;
                const char* va = vpool + ((int64_t)pg * p.v_batch + (int64_t)pr * p.v_row) * esz;
                if (kv8) {
                    const uint2 kx = *reinterpret_cast<const uint2*>(ka);
                    const uint2 vx = *reinterpret_cast<const uint2*>(va);
                    ko[i] = ok ? fp8x8_to<T>(kx.x, kx.y, p.k_scale) : u32x4{0, 0, 0, 0};
                    vo[i] = ok ? fp8x8_to<T>(vx.x, vx.y, p.v_scale) : u32x4{0, 0, 0, 0};
                } else {
                    const u32x4 kx = *reinterpret_cast<const u32x4*>(ka);
                    const u32x4 vx = *reinterpret_cast<const u32x4*>(va);
                    ko[i] = ok ? kx : u32x4{0, 0, 0, 0};
                    vo[i] = ok ? vx : u32x4{0, 0, 0, 0};
                }
            } else if (kv8) {
                const u32x2 kx = buf_load8(krs, ok ? n * (int)p.k_row + lc * 8 : kOOB);
                const u32x2 vx = buf_load8(vrs, ok ? n * (int)p.v_row + lc * 8 : kOOB);
                ko[i] = fp8x8_to<T>(kx[0], kx[1], p.k_scale);
                vo[i] = fp8x8_to<T>(vx[0], vx[1], p.v_scale);
            } else {
                ko[i] = buf_load16(krs, ok ? n * (int)p.k_row * 2 + lc * 16 : kOOB);
                vo[i] = buf_load16(vrs, ok ? n * (int)p.v_row * 2 + lc * 16 : kOOB);
            }
        }
    };
    auto store_from = [&](int buf, const u32x4 (&ki)[NLD], const u32x4 (&vi)[NLD]) {
        char* ks = smem + buf * TILE;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int r = lrow0 + i * LROW_STEP;
            *reinterpret_cast<u32x4*>(ks + kv_off<HD>(r, lc)) = ki[i];
            *reinterpret_cast<u32x4*>(ks + VREG + kv_off<HD>(r, lc)) = vi[i];
        }
    };

    // Per-lane LDS read addresses (kv_off image): the K row read of k-step s, 32-key half kt
    // is kb[s & 1] + RB*4*kt + 512*(s >> 1) (RB = bytes of an 8-row block); the V^T transposed
    // read (kt, sp, dt, part) is vb[part] + RB*(4 kt + 2 sp) + 512 dt.  Everything but the
    // two base registers of each operand is an immediate offset of the ds_read.
    constexpr int RB = HD * 16;                 // bytes of one 8-row block of the image
    const int q4 = (lane & 15) >> 2;
    int kb[2], vb[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        kb[u] = (int)(size_t)smem + kv_off<HD>(lr, 2 * u + hh);
        const int r = 8 * u + 4 * hh + q4;
        const int col = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        vb[u] = (int)(size_t)smem + VREG + kv_off<HD>(r, col >> 3) + 8 * ((col >> 2) & 1);
    }
    typedef __attribute__((address_space(3))) V8 lds_v8;
    f32x16 acc_o[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) acc_o[dt] = f32x16{};
    // running row max in scaled (log2) units: P = exp2(S c - m_sc); -inf until the row's first
    // visible key
    float m_sc = -INFINITY;
    float l_run = 0.f;

    // ---- the pieces of one 64-key tile
    // K operand of S^T = K Q^T for k-step s, 32-key half `kt`, read row-wise from the LDS image
    // of buffer `buf`
    auto rd_k = [&](const int buf, const int s, const int kt) {
        return *(const lds_v8*)(size_t)(kb[s & 1] + buf * TILE + kt * 4 * RB + 512 * (s >> 1));
    };
    // V^T operand of O^T += V^T P^T for (kt, sp, dt) through the transposing LDS read
    auto rd_v = [&](const int buf, const int i) {
        const int kt = i / (2 * ND), sp = (i / ND) & 1, dt = i % ND;
        const int o = buf * TILE + (4 * kt + 2 * sp) * RB + 512 * dt;
        const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(vb[0] + o));
        const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(vb[1] + o));
        const s16x8 av = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
        return __builtin_bit_cast(V8, av);
    };
    // score transforms of values [v0, v0 + n) (flattened st[kt][r], v = 16 kt + r); masking
    // only where a window edge crosses the tile
    auto transform_part = [&](f32x16 (&st)[2], const int n0, const bool need_mask, const int v0,
                              const int n) {
#pragma unroll
        for (int v = v0; v < v0 + n; ++v) {
            const int kt = v >> 4, r = v & 15;
            const int key = n0 + 4 * hh + 32 * kt + (r & 3) + 8 * (r >> 2);
            if (FEAT && p.softcap_pre > 0.f) st[kt][r] = fast_tanh(st[kt][r] * p.softcap_pre);
            if (FEAT && p.alibi) st[kt][r] -= alibi_w * (float)abs(pos + diag - key);
            if (need_mask && (key >= my_lr || key < my_ll)) st[kt][r] = -INFINITY;
        }
    };
    // Deferred rescale: the running max m_sc (the exp reference) only moves once some row's
    // true max exceeds it by more than max_slack (log2 units), so P = exp2(S c - m_sc) stays
    // below 2^max_slack; O, l and the LSE are all relative to the same m_sc, so the result is
    // unchanged up to rounding (the relative rounding of P in T does not depend on the scale).
    auto rescale_o = [&](const float alpha) {
        l_run *= alpha;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc_o[dt][r] *= alpha;
    };
    auto raise_max = [&](const float mx) {
        const float m_new = fmaxf(m_sc, mx * c);
        if (__any(m_new > m_sc + p.max_slack)) {
            rescale_o(m_new == -INFINITY ? 1.f : fast_exp2(m_sc - m_new));
            m_sc = m_new;
        }
    };
    // P = exp2(S c - m c) -> T (the B operand of the PV product) for values [v0, v0 + n);
    // the row sum accumulates the fp32 P values, as the reference's softmax does
    // (softmax_hip.h:129-189), so the LSE is the fp32 log-sum-exp of the scores.  (Summing the
    // rounded bf16 pairs with v_dot2c instead costs ~14 cycles a pair beside the MFMAs and moves
    // the LSE by up to the bf16 unit roundoff, 2^-9; the fp32 adds fit the register budget only
    // with the two-base kv_off image.)
    typedef __attribute__((ext_vector_type(2))) float f2;
    typedef typename DT<T>::v2 T2;
    auto exp_part = [&](const f32x16 (&st)[2], V8 (&pb)[4], const f2 m2, float (&rs)[2],
                        const int v0, const int n) {
        const f2 c2 = {c, c};
#pragma unroll
        for (int v = v0; v < v0 + n; v += 2) {
            const int kt = v >> 4, r = v & 15;
            f2 x = {st[kt][r], st[kt][r + 1]};
            x = __builtin_elementwise_fma(x, c2, -m2);
            const float e0 = fast_exp2(x[0]), e1 = fast_exp2(x[1]);
            rs[0] += e0;
            rs[1] += e1;
            const T2 e = {(T)e0, (T)e1};
            pb[2 * kt + (r >> 3)][r & 7] = e[0];
            pb[2 * kt + (r >> 3)][(r & 7) + 1] = e[1];
        }
    };
    // dropout on the P operand of PV (the row sums keep the undropped P, as the reference's
    // softmax does before apply_dropout, flash_fwd_kernel_hip.h): each run of 4 keys of this
    // lane's row draws one Philox block (fmha_common.h drop_block)
    auto drop_tile = [&](V8 (&pb)[4], const int n0) {
        if (!(FEAT && p.drop)) return;
        const int bhg = bidx * p.h + head;
        uint64_t dseed, doff;
        drop_key(p, dseed, doff);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32x4 w = drop_block(dseed, doff, bhg, pos, n0 + 32 * kt + 8 * j + 4 * hh);
                const uint32_t word = (pos & 2) ? ((pos & 1) ? w[3] : w[2]) : ((pos & 1) ? w[1] : w[0]);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (!drop_keep(word, i, p.keep_thr)) pb[2 * kt + (j >> 1)][(j & 1) * 4 + i] = (T)0.f;
            }
    };
    auto exp_ref = [&]() {
        const float mref = (m_sc == -INFINITY) ? 0.f : m_sc;
        return f2{mref, mref};
    };
    // S^T = K Q^T (LDS reads one k-step ahead of the MFMAs)
    auto qk = [&](const int ks, f32x16 (&st)[2]) {
        st[0] = f32x16{};
        st[1] = f32x16{};
        V8 a0 = rd_k(ks, 0, 0), a1 = rd_k(ks, 0, 1);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            V8 n0 = a0, n1 = a1;
            if (s + 1 < NS) { n0 = rd_k(ks, s + 1, 0); n1 = rd_k(ks, s + 1, 1); }
            st[0] = DT<T>::mfma32(a0, qf[s], st[0]);
            st[1] = DT<T>::mfma32(a1, qf[s], st[1]);
            a0 = n0;
            a1 = n1;
        }
    };
    // O^T += V^T P^T (V^T reads one MFMA ahead)
    constexpr int NPV = 4 * ND;                 // PV MFMAs per tile
    auto pv = [&](const int vs, const V8 (&pb)[4]) {
        V8 a = rd_v(vs, 0);
#pragma unroll
        for (int i = 0; i < NPV; ++i) {
            V8 nx = a;
            if (i + 1 < NPV) nx = rd_v(vs, i + 1);
            acc_o[i % ND] = DT<T>::mfma32(a, pb[i / ND], acc_o[i % ND]);
            a = nx;
        }
    };
    auto row_max = [&](const f32x16 (&st)[2]) {
        float mx = st[0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, st[0][r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[1][r]);
        return wave_max_halves(mx);
    };
    auto exp_tile = [&](const f32x16 (&st)[2], V8 (&pb)[4]) {
        float rs[2] = {0.f, 0.f};
        exp_part(st, pb, exp_ref(), rs, 0, 32);
        l_run += rs[0] + rs[1];
    };
    // The pipeline's scores are X = S c - m_sc already: P = exp2(X) -> T for values [v0, v0 + n)
    auto expx_part = [&](const f32x16 (&st)[2], V8 (&pb)[4], float& rs, const int v0, const int n) {
#pragma unroll
        for (int v = v0; v < v0 + n; v += 2) {
            const int kt = v >> 4, r = v & 15;
            const float e0 = fast_exp2(st[kt][r]), e1 = fast_exp2(st[kt][r + 1]);
            rs += e0;
            rs += e1;
            const T2 e = {(T)e0, (T)e1};
            pb[2 * kt + (r >> 3)][r & 7] = e[0];
            pb[2 * kt + (r >> 3)][(r & 7) + 1] = e[1];
        }
    };
    auto expx_tile = [&](const f32x16 (&st)[2], V8 (&pb)[4]) {
        float rs = 0.f;
        expx_part(st, pb, rs, 0, 32);
        l_run += rs;
    };
    // Deferred rescale on pipeline scores: mx = this row's max of X = S c - m_sc over the new
    // tile.  Rows still at m_sc = -inf had X computed against 0 (exp_ref) and take m_sc = mx.
    auto rescale_x = [&](const float mx, f32x16 (&sx)[2]) {
        const bool fresh = m_sc == -INFINITY;
        if (__any(mx > p.max_slack || (fresh && mx != -INFINITY))) {
            // a volatile asm cannot be speculated: keeps the rare rescale a real branch
            // (if-converted it costs 64 VALU on every tile)
            asm volatile("; rescale_x");
            const float delta = fresh ? (mx == -INFINITY ? 0.f : mx) : fmaxf(mx, 0.f);
            rescale_o(fresh ? 1.f : fast_exp2(-delta));
#pragma unroll
            for (int v = 0; v < 32; ++v) sx[v >> 4][v & 15] -= delta;
            m_sc = fresh ? (mx == -INFINITY ? -INFINITY : mx) : m_sc + delta;
        }
    };

    // ---- tiles that need per-wave masking / skipping: one tile in flight, two LDS buffers
    auto masked_range = [&](const int lo, const int hi) {
        if (lo >= hi) return;
        load_to(lo, kr, vr);
        store_from(0, kr, vr);
        // Retire every outstanding load (Q fragments included) here: otherwise the loop-header
        // merge of the waitcnt scoreboard makes the first QK^T MFMA of EVERY iteration wait
        // vmcnt(0), i.e. drain the next tile's prefetch (vmcnt=0, expcnt=7, lgkmcnt=15).
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
        int buf = 0;
        for (int nb = lo; nb < hi; ++nb) {
            const bool more = nb + 1 < hi;
            if (more) load_to(nb + 1, kr, vr);
            const int n0 = nb * kBlockN;
            const bool active = wave_ok && n0 < w_lr_max && n0 + kBlockN > w_ll_min;
            if (active) {
                f32x16 st[2];
                qk(buf, st);
                transform_part(st, n0, (n0 + kBlockN > w_lr_min) || (n0 < w_ll_max), 0, 32);
                raise_max(row_max(st));
                V8 pb[4];
                exp_tile(st, pb);
                drop_tile(pb, n0);
                pv(buf, pb);
            }
            if (more) store_from(buf ^ 1, kr, vr);
            __syncthreads();
            buf ^= 1;
        }
    };

    // V^T operand through inline-asm transposing reads: the compiler's waitcnt pass treats
    // the ds_read_tr builtin as aliasing every in-flight LDS-DMA and would drain the DMA queue
    // (vmcnt(0)) before it; the asm reads are covered by explicit lgkmcnt waits instead.
    // Byte offset OFF (buffer + row block) is an immediate.
    auto rd_v_asm = [&](auto OFF) {
        constexpr int off = decltype(OFF)::value;
        s16x4 t0, t1;
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(t0) : "v"(vb[0]), "i"(off));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(t1) : "v"(vb[1]), "i"(off));
        const s16x8 av = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
        return __builtin_bit_cast(V8, av);
    };
    auto lgkm_wait = [&](auto N) {
        constexpr int n = decltype(N)::value;
        __builtin_amdgcn_s_waitcnt(0xC07F | (n << 8));
        // the MFMA consuming the asm-read registers must not be scheduled above the wait
        __builtin_amdgcn_sched_barrier(0);
    };

    // ---- tiles every row of the workgroup sees in full: two-stage software pipeline.
    // Step j issues QK^T of tile j+1 beside the softmax VALU of tile j, then PV of tile j beside
    // the row max of tile j+1 (T15): the MFMA pipe always has independent work while the VALU
    // finishes a tile.  K/V tiles stream straight into LDS (buffer_load ... lds, no staging
    // registers) three tiles ahead through NBUF = 4 rotating buffers: at step j buffer
    // (j+1)%4 holds K of j+1, j%4 holds V of j, and tiles j+2 (landing) and j+3 (issued now)
    // are in flight.  One raw s_barrier per tile, preceded by a counted vmcnt that retires
    // exactly tile j+2.  The LDS image is the same swizzled image the register-staged path
    // writes: lane l of a wave-instruction lands at +16 l, so it fetches the global chunk
    // (l % CPR) ^ swz(row) of its row.
    constexpr int IPW = TILE / 1024 / NW;          // DMA wave-instructions per wave per K (V) tile
    static_assert(IPW >= 1 && IPW * 1024 * NW == TILE, "DMA geometry");
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    int dma_k[IPW], dma_v[IPW];                    // per-lane byte offsets within a tile
    constexpr int PPB = CPR / 8;                   // DMA pieces per 8-row block
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
        // piece g = 8 rows x 8 chunks of the kv_off image: lane l lands at g KiB + 16 l
        const int g = wave * IPW + i;
        const int r = 8 * (g / PPB) + (lane & 31) / 4;
        const int cch = 8 * (g % PPB) + 4 * (lane >> 5) + ((lane & 3) ^ ((r >> 2) & 3));
        const bool ok = cch * 8 < p.d;
        dma_k[i] = ok ? r * (int)p.k_row * 2 + cch * 16 : kOOB;
        dma_v[i] = ok ? r * (int)p.v_row * 2 + cch * 16 : kOOB;
    }
    typedef __attribute__((address_space(3))) void lds_void;
    auto dma_tile = [&](const int nb, const int buf) {
        // (soffset pinned to an SGPR: derived from a tile index the compiler kept in a VGPR,
        // each DMA piece became a waterfall loop)
        const int kso = __builtin_amdgcn_readfirstlane(nb * kBlockN * (int)p.k_row * 2);
        const int vso = __builtin_amdgcn_readfirstlane(nb * kBlockN * (int)p.v_row * 2);
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int g = wave_u * IPW + i;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                krs, (lds_void*)(smem + buf * TILE + g * 1024), 16, dma_k[i], kso, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                vrs, (lds_void*)(smem + VREG + buf * TILE + g * 1024), 16, dma_v[i], vso, 0, 0);
        }
    };
    // counted vmcnt (the DMA writes are invisible to the compiler's waitcnt tracking) + a
    // barrier that the compiler may not move memory operations across
    constexpr int NDMA = 2 * IPW;                  // vmem instructions per tile per wave
    auto publish = [&](const bool one_in_flight) {
        if (one_in_flight) __builtin_amdgcn_s_waitcnt(waitcnt_vm(NDMA));
        else __builtin_amdgcn_s_waitcnt(0x0F70);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // D = 256 (no pipeline, NBUF = 2): the per-wave masked loop with K/V by LDS-DMA, tile
    // j+1 in flight while tile j computes (no staging registers: the 512-register budget is
    // taken by the Q fragments and the O accumulator)
    auto dma_range = [&](const int lo, const int hi) {
        if (lo >= hi) return;
        dma_tile(lo, 0);
        publish(false);
        int buf = 0;
        for (int nb = lo; nb < hi; ++nb) {
            if (nb + 1 < hi) dma_tile(nb + 1, buf ^ 1);
            const int n0 = nb * kBlockN;
            const bool active = wave_ok && n0 < w_lr_max && n0 + kBlockN > w_ll_min;
            if (active) {
                f32x16 st[2];
                qk(buf, st);
                transform_part(st, n0, (n0 + kBlockN > w_lr_min) || (n0 < w_ll_max), 0, 32);
                raise_max(row_max(st));
                V8 pb[4];
                exp_tile(st, pb);
                drop_tile(pb, n0);
                pv(buf, pb);
            }
            publish(false);
            buf ^= 1;
        }
    };
    // Tiles [lo, hm) need no mask; tiles [hm, hi) (the causal diagonal / right window edge /
    // ragged end) are masked in registers on the way through the same pipeline (a wave whose
    // rows cannot see such a tile computes zeros for it instead of branching out of the
    // interleaved schedule).  Every row sees tile lo (f_lo lies past every row's left window
    // edge, and visible keys are contiguous), so only the right edge can cut a pipeline tile.
    //
    // Scores leave phase b already scaled and shifted, X = S c - m_sc, so phase a is exp + cvt
    // only; the VALU of a tile splits evenly between the two MFMA phases (per wave and tile:
    // a = 32 v_exp + 32 fp32 row-sum adds + 16 cvt beside 16 QK^T MFMAs, b = 32 fma + 16 max3
    // beside 16 PV MFMAs), each within the MFMA gaps.  The edge mask runs after phase b on the edge tiles only.
    const int lim_e = my_lr - 4 * hh;            // right edge of this lane's keys, minus its offset
    auto pipe_range = [&](const int lo, const int hm, const int hi) {
        const bool third = lo + 2 < hi;
        dma_tile(lo, 0);
        dma_tile(lo + 1, 1);
        if (third) dma_tile(lo + 2, 2);
        publish(third);
        // scores ping-pong between sa and sb from step to step (st: this tile, sn: the next),
        // so the QK^T accumulators never need a register copy onto a loop-carried value
        f32x16 sa[2], sb[2];
        qk(0, sa);
        transform_part(sa, lo * kBlockN, lo >= hm, 0, 32);
        raise_max(row_max(sa));
        {
            const float mr = exp_ref()[0];
#pragma unroll
            for (int v = 0; v < 32; ++v) sa[v >> 4][v & 15] = __builtin_fmaf(sa[v >> 4][v & 15], c, -mr);
        }
        const int nsteps = hi - lo - 1;
        auto step = [&](auto KB, auto VB, auto WB, const int j, f32x16 (&st)[2], f32x16 (&sn)[2]) {
            constexpr int ks = decltype(KB)::value, vs = decltype(VB)::value, wb = decltype(WB)::value;
            const bool issue = j + 3 < hi;
            if (issue) dma_tile(j + 3, wb);
            if (SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);
            // phase a: S_{j+1} = K_{j+1} Q^T on the MFMA pipe, P_j = exp2(X_j) -> T on the VALU
            sn[0] = f32x16{};
            sn[1] = f32x16{};
            V8 pb[4];
            float rs = 0.f;                       // fp32 row sum of P_j
            constexpr int EV = 32 / (2 * NS);     // exp values per QK^T MFMA
            V8 a0 = rd_k(ks, 0, 0), a1 = rd_k(ks, 0, 1);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                V8 n0 = a0, n1 = a1;
                if (s + 1 < NS) { n0 = rd_k(ks, s + 1, 0); n1 = rd_k(ks, s + 1, 1); }
                sn[0] = DT<T>::mfma32(a0, qf[s], sn[0]);
                expx_part(st, pb, rs, (2 * s) * EV, EV);
                sn[1] = DT<T>::mfma32(a1, qf[s], sn[1]);
                expx_part(st, pb, rs, (2 * s + 1) * EV, EV);
                // pins the row-sum adds into this MFMA gap: unpinned, the compiler sinks them
                // below phase b (rs is only read there) into a VALU-only run of 32 adds
                // (+1.5-2 % C2, same-box A/B)
                asm volatile("" : "+v"(rs));
                a0 = n0;
                a1 = n1;
                if (SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);
            }
            // phase b: O += V_j^T P_j on the MFMA pipe; on the VALU X_{j+1} = S_{j+1} c - m_sc
            // (transforms and edge mask first) and its row max; V^T read two MFMAs ahead (asm
            // reads, explicit lgkmcnt)
            constexpr int MV = 32 / NPV;          // score values per PV MFMA
            auto voffs = [&](auto I) {             // immediate offset of PV operand I
                constexpr int i = decltype(I)::value;
                return std::integral_constant<int, vs * TILE + (4 * (i / (2 * ND)) + 2 * ((i / ND) & 1)) * RB + 512 * (i % ND)>{};
            };
            const float mr = exp_ref()[0];
            float mx = -INFINITY;
            V8 ring[3];
            ring[0] = rd_v_asm(voffs(std::integral_constant<int, 0>{}));
            ring[1] = rd_v_asm(voffs(std::integral_constant<int, 1>{}));
            static_for<NPV>([&](auto I) {
                constexpr int i = decltype(I)::value;
                if constexpr (i + 2 < NPV) {
                    ring[(i + 2) % 3] = rd_v_asm(voffs(std::integral_constant<int, i + 2>{}));
                    lgkm_wait(std::integral_constant<int, 4>{});
                } else if constexpr (i + 1 < NPV) {
                    lgkm_wait(std::integral_constant<int, 2>{});
                } else {
                    lgkm_wait(std::integral_constant<int, 0>{});
                }
                acc_o[i % ND] = DT<T>::mfma32(ring[i % 3], pb[i / ND], acc_o[i % ND]);
                if (FEAT) transform_part(sn, (j + 1) * kBlockN, false, i * MV, MV);
#pragma unroll
                for (int v = i * MV; v < (i + 1) * MV; ++v)
                    sn[v >> 4][v & 15] = __builtin_fmaf(sn[v >> 4][v & 15], c, -mr);
                if constexpr (MV == 2) mx = fmaxf(fmaxf(mx, sn[(i * 2) >> 4][(i * 2) & 15]), sn[(i * 2 + 1) >> 4][(i * 2 + 1) & 15]);
                else {
#pragma unroll
                    for (int v = i * MV; v < (i + 1) * MV; ++v) mx = fmaxf(mx, sn[v >> 4][v & 15]);
                }
                if (SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);
            });
            // an opaque use pins the max chain inside phase b (else it is sunk below the edge
            // branch, out of the MFMA gaps)
            asm volatile("" : "+v"(mx));
            l_run += rs;
            if (j + 1 >= hm) {                    // edge tile: mask, then the row max again
                const int lim_t = lim_e - (j + 1) * kBlockN;
                float mm = -INFINITY;
#pragma unroll
                for (int v = 0; v < 32; ++v) {
                    const int off = 32 * (v >> 4) + ((v & 15) & 3) + 8 * ((v & 15) >> 2);
                    if (off >= lim_t) sn[v >> 4][v & 15] = -INFINITY;
                    mm = fmaxf(mm, sn[v >> 4][v & 15]);
                }
                mx = mm;
            }
            // the decision needs no row max: some lane's half-row max passes the slack iff some
            // row's does, so the halves are combined only on the (rare) rescale path
            if (__any(mx > p.max_slack || (m_sc == -INFINITY && mx != -INFINITY)))
                rescale_x(wave_max_halves(mx), sn);
            publish(issue);                       // tile j+2 landed everywhere
        };
        typedef std::integral_constant<int, 0> I0;
        typedef std::integral_constant<int, 1> I1;
        typedef std::integral_constant<int, 2> I2;
        typedef std::integral_constant<int, 3> I3;
        // step r (tile j = lo + r) reads K of j+1 from buffer (r+1)%4 and V of j from r%4.
        // Causal diagonal / right window edge: a wave stops after the last tile any of its rows
        // sees (visible keys are contiguous) — drains it, then only issues its DMA share and
        // joins the barriers for the rest of the workgroup's steps (the same barrier count).
        // The skipped tiles would add exact zeros, so results are bit-identical, and the
        // wave's SIMD partner gets the whole issue port meanwhile.
        const int t_w = __builtin_amdgcn_readfirstlane((w_lr_max + kBlockN - 1) / kBlockN - 1);
        const int nsteps_w = __builtin_amdgcn_readfirstlane(wave_ok ? max(0, min(nsteps, t_w - lo)) : nsteps);
        int r = 0;
        while (r < nsteps_w) {
            step(I1{}, I0{}, I3{}, lo + r, sa, sb);
            if (++r >= nsteps_w) break;
            step(I2{}, I1{}, I0{}, lo + r, sb, sa);
            if (++r >= nsteps_w) break;
            step(I3{}, I2{}, I1{}, lo + r, sa, sb);
            if (++r >= nsteps_w) break;
            step(I0{}, I3{}, I2{}, lo + r, sb, sa);
            ++r;
        }
        // drain: the wave's last tile's softmax and PV.  V^T through the asm reads: a wave that
        // leaves early still has its DMA share of tile j+3 in flight, and the builtin
        // transposing read would make the compiler drain it (vmcnt(0)) first
        V8 pb[4];
        if (nsteps_w & 1) expx_tile(sb, pb);
        else expx_tile(sa, pb);
        auto pv_asm = [&](auto VB) {
            constexpr int vs = decltype(VB)::value;
            auto voffs = [&](auto I) {
                constexpr int i = decltype(I)::value;
                return std::integral_constant<int, vs * TILE + (4 * (i / (2 * ND)) + 2 * ((i / ND) & 1)) * RB + 512 * (i % ND)>{};
            };
            V8 ring[3];
            ring[0] = rd_v_asm(voffs(std::integral_constant<int, 0>{}));
            ring[1] = rd_v_asm(voffs(std::integral_constant<int, 1>{}));
            static_for<NPV>([&](auto I) {
                constexpr int i = decltype(I)::value;
                if constexpr (i + 2 < NPV) {
                    ring[(i + 2) % 3] = rd_v_asm(voffs(std::integral_constant<int, i + 2>{}));
                    lgkm_wait(std::integral_constant<int, 4>{});
                } else if constexpr (i + 1 < NPV) {
                    lgkm_wait(std::integral_constant<int, 2>{});
                } else {
                    lgkm_wait(std::integral_constant<int, 0>{});
                }
                acc_o[i % ND] = DT<T>::mfma32(ring[i % 3], pb[i / ND], acc_o[i % ND]);
            });
        };
        switch (nsteps_w & 3) {
            case 0: pv_asm(I0{}); break;
            case 1: pv_asm(I1{}); break;
            case 2: pv_asm(I2{}); break;
            default: pv_asm(I3{}); break;
        }
        // the steps this wave skips: its DMA share and the barriers only
        for (; r < nsteps; ++r) {
            const int j = lo + r;
            const bool issue = j + 3 < hi;
            if (issue) dma_tile(j + 3, (r + 3) & 3);
            publish(issue);
        }
        __syncthreads();
    };
    // Key tiles: [nb_lo, f_lo) cross the left window edge (per-wave masked loop);
    // [f_lo, f_hi) every row of the workgroup sees in full; [f_hi, nb_hi) cross the right
    // window edge / the end of the keys.  The last two ranges run through the pipeline.
    int f_lo = nb_hi, f_hi = nb_hi;
    if (PIPE && p.pipe && !paged && !kv8 && !(FEAT && p.drop)) {
        const int ll_max = lim_l(pos_hi), lr_min = lim_r(pos_lo);
        f_lo = max(nb_lo, (ll_max + kBlockN - 1) / kBlockN);
        f_hi = max(f_lo, min(nb_hi, lr_min / kBlockN));
        if (nb_hi - f_lo < 2 || (p.pipe == 2 && f_hi - f_lo < 2)) f_lo = f_hi = nb_hi;
    }
    if (p.prio_hi && __builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);
    // (fwd_pipe=2: edge tiles through the per-wave masked loop instead - A/B knob)
    const int p_hi = (p.pipe == 2 && f_hi - f_lo >= 2) ? f_hi : nb_hi;
    if (!PIPE && !paged && !kv8) dma_range(nb_lo, f_lo);
    else masked_range(nb_lo, f_lo);
    if constexpr (PIPE) {
        if (f_lo < p_hi) pipe_range(f_lo, f_hi, p_hi);
    }
    masked_range(p_hi, nb_hi);

    // ---- epilogue: normalise, write O (or the split partial) and LSE
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
        if (hh == 0) p.lseaccum[rid] = empty ? -INFINITY : (m_sc + __log2f(l_full)) * kLn2;
        return;
    }
    T* orow = reinterpret_cast<T*>(p.o) + (int64_t)bidx * p.o_batch +
              (int64_t)(q_off + pos) * p.o_row + (int64_t)head * p.o_head;
    store_o_row16<T, ND>(orow, acc_o, (FEAT && p.drop) ? inv * p.rp_keep : inv, p.d, hh);
    if (p.lse && hh == 0) {
        p.lse[(int64_t)bidx * p.lse_batch + (int64_t)head * p.lse_head + q_off + pos] =
            empty ? INFINITY : (m_sc + __log2f(l_full)) * kLn2;
    }
}

// Grid: either one workgroup per item (grid = (b*hk, m_blocks, splits), heaviest causal row
// blocks dispatched first), or persistent (p.persistent: grid = (resident workgroups, 1,
// splits)), each workgroup walking items in a heaviest-first boustrophedon order so the
// causal work per workgroup balances, and one item's O-store tail overlaps the next item's
// prologue loads instead of a workgroup boundary.
template <int HD, typename T, int NW, bool MASK, bool FEAT>
__global__ void __launch_bounds__(NW * 64, fwd_waves_per_simd(HD)) fmha_fwd_kernel(const FwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int s_claim[2];
    const int nbh = p.b * p.hk;
    const int g = gridDim.x;
    for (int k = 0;; ++k) {        // one call site: the item body is inlined once
        int bh, m_block;
        if (p.persistent == 2) {
            // XCD-grouped pairs: pair i of (b, kv head) = row blocks (n-1-i, i), equal causal
            // work; consecutive pairs of one (b, kv head) run at the same time on the CUs of
            // one XCD (workgroup bid sits on XCD bid % 8), so they share that XCD's L2 for K/V
            const int nm = p.n_mblocks, npair = (nm + 1) >> 1;
            const int bid = (int)blockIdx.x;
            const int v = (bid & 7) * (g >> 3) + (bid >> 3);
            const int q = (k >> 1) * g + v;
            if (q >= nbh * npair) break;
            bh = q / npair;
            const int i = q - bh * npair;
            m_block = (k & 1) ? i : nm - 1 - i;
            if ((k & 1) && i == nm - 1 - i) continue;   // odd count: the middle block is alone
        } else if (p.persistent == 3) {
            // dynamic queue: claim the next item (heaviest row block first, then (b, kv head))
            // from a device counter, so ragged varlen items balance as workgroups finish; the
            // claim slot alternates so a fast wave's next claim cannot overwrite it unread
            // p.xcd_queues (default): one queue per XCD over the units bh = x (mod 8), unit-major,
            // so a unit's row blocks run together on one XCD and share its L2 for K/V (workgroup
            // b sits on XCD b % 8; slots % 8 == 0 and nbh >= 8 are checked on the host)
            const int x = p.xcd_queues ? (int)(blockIdx.x & 7) : 0;
            const int nq = p.xcd_queues ? (nbh - x + 7) >> 3 : nbh;
            if (threadIdx.x == 0) s_claim[k & 1] = atomicAdd(p.work_ctr + 2 + x, 1);
            __syncthreads();
            const int q = s_claim[k & 1];
            if (q >= nq * p.n_mblocks) break;
            if (p.xcd_queues) {     // unit-major: an XCD's workgroups share a unit's K/V in L2
                bh = x + 8 * (q / p.n_mblocks);
                m_block = p.n_mblocks - 1 - q % p.n_mblocks;
            } else {                // heaviest row block first over all units
                bh = q % nq;
                m_block = p.n_mblocks - 1 - q / nq;
            }
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
        fwd_item<HD, T, NW, MASK, FEAT>(p, smem, bh, m_block, blockIdx.z);
    }
    // the key this launch used, for the backward (the reference writes params.rng_state the
    // same way, flash_fwd_kernel_hip.h); one lane of one workgroup
    if (FEAT && p.drop && p.rng_out && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 &&
        threadIdx.x == 0) {
        uint64_t dseed, doff;
        drop_key(p, dseed, doff);
        p.rng_out[0] = (int64_t)dseed;
        p.rng_out[1] = (int64_t)doff;
    }
    // dynamic queue: every workgroup has made its last (failed) claim when it gets here; the
    // last one to finish resets the counters for the next launch on this stream
    if (p.persistent == 3 && threadIdx.x == 0) {
        const int total = (int)(gridDim.x * gridDim.y * gridDim.z);
        if (atomicAdd(p.work_ctr + 1, 1) == total - 1) {
            for (int i = 2; i < 10; ++i) atomicExch(p.work_ctr + i, 0);
            atomicExch(p.work_ctr + 1, 0);
        }
    }
}

// Split-KV combine: lse = log sum_s exp(lse_s); O = sum_s exp(lse_s - lse) O_s
// (reference combine_attn_seqk_parallel, flash_fwd_kernel_hip.h:1322-1568; empty -> +inf).
// One wave per (b, h, pos) row.
template <int HD, typename T>
__global__ void __launch_bounds__(256) fmha_combine_kernel(const CombineParams cp) {
    // The split partials are independent loads: the LSE reduction runs with the splits across
    // the lanes, and the O sum keeps CU = 8 splits' rows in flight per wave (a serial loop over
    // splits exposes one load latency per split, which at 32 splits cost more than the bytes).
    const int lane = threadIdx.x & 63;
    const int64_t rid = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t rows = (int64_t)cp.b * cp.h * cp.seqlen_q;
    if (rid >= rows) return;
    const int pos = (int)(rid % cp.seqlen_q);
    const int head = (int)((rid / cp.seqlen_q) % cp.h);
    const int bidx = (int)(rid / ((int64_t)cp.seqlen_q * cp.h));
    const int ns = cp.dec_ns ? cp.dec_ns[bidx] : cp.num_splits;
    float mx = -INFINITY;
    for (int s = lane; s < ns; s += 64) mx = fmaxf(mx, cp.lseaccum[s * rows + rid]);
    mx = wave_max_halves(mx);
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    float sum = 0.f;
    if (mx != -INFINITY)
        for (int s = lane; s < ns; s += 64) sum += __expf(cp.lseaccum[s * rows + rid] - mx);
    sum = wave_sum_halves(sum);
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) sum += __shfl_xor(sum, off);
    const bool empty = (mx == -INFINITY) || sum == 0.f;
    const float lse = empty ? INFINITY : __logf(sum) + mx;
    constexpr int PER = HD / 64;
    constexpr int CU = 8;
    typedef float __attribute__((ext_vector_type(PER))) fv;
    fv acc = {};
    if (!empty) {
        const float* oa = cp.oaccum + rid * HD + lane * PER;
        const int64_t sstride = rows * HD;
        int s = 0;
        for (; s + CU <= ns; s += CU) {
            fv x[CU];
            float w[CU];
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                x[u] = *reinterpret_cast<const fv*>(oa + (s + u) * sstride);
                w[u] = __expf(cp.lseaccum[(s + u) * rows + rid] - lse);
            }
#pragma unroll
            for (int u = 0; u < CU; ++u) acc += w[u] * x[u];
        }
        for (; s < ns; ++s)
            acc += __expf(cp.lseaccum[s * rows + rid] - lse) * *reinterpret_cast<const fv*>(oa + s * sstride);
    }
    T* orow = reinterpret_cast<T*>(cp.o) + (int64_t)bidx * cp.o_batch + (int64_t)pos * cp.o_row +
              (int64_t)head * cp.o_head;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int d = lane * PER + i;
        if (d < cp.d) orow[d] = (T)acc[i];
    }
    if (cp.lse && lane == 0)
        cp.lse[(int64_t)bidx * cp.lse_batch + (int64_t)head * cp.lse_head + pos] = lse;
}

// Split-KV combine, one workgroup per row (few rows: the decode shapes, where the per-wave kernel
// above leaves most CUs idle and waits one memory latency per batch of 8 splits).  Thread t owns
// float4 chunk t % (HD / 4) of the splits s = t / (HD / 4) (mod 256 / (HD / 4)): every partial
// row of the first 8 rounds is loaded before the LSE merge (wave 0, splits across lanes) has
// produced the weights, so the row costs about one memory latency; the 256 / (HD / 4) partial
// sums of a chunk meet in LDS.  HD in {64, 128, 256}, at most 128 splits.
template <int HD, typename T>
__global__ void __launch_bounds__(256) fmha_combine_row_kernel(const CombineParams cp) {
    constexpr int D4 = HD / 4;
    constexpr int G = 256 / D4;
    constexpr int NB = 8;
    static_assert(G * D4 == 256, "chunks per thread");
    __shared__ float wsh[128];
    __shared__ f32x4 red[G][D4];
    const int t = threadIdx.x;
    const int64_t rid = blockIdx.x;
    const int64_t rows = (int64_t)cp.b * cp.h * cp.seqlen_q;
    const int pos = (int)(rid % cp.seqlen_q);
    const int head = (int)((rid / cp.seqlen_q) % cp.h);
    const int bidx = (int)(rid / ((int64_t)cp.seqlen_q * cp.h));
    const int ns = cp.dec_ns ? cp.dec_ns[bidx] : cp.num_splits;
    const int c = t % D4, g = t / D4;
    const float* oa = cp.oaccum + rid * HD + 4 * c;
    const int64_t sstride = rows * HD;
    f32x4 x[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int sp = g + G * u;
        x[u] = sp < ns ? *reinterpret_cast<const f32x4*>(oa + sp * sstride) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (t < 64) {
        const float l0 = t < ns ? cp.lseaccum[t * rows + rid] : -INFINITY;
        const float l1 = t + 64 < ns ? cp.lseaccum[(t + 64) * rows + rid] : -INFINITY;
        float mx = wave_max_halves(fmaxf(l0, l1));
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
        float sum = mx == -INFINITY ? 0.f : __expf(l0 - mx) + __expf(l1 - mx);
        sum = wave_sum_halves(sum);
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) sum += __shfl_xor(sum, off);
        const bool empty = (mx == -INFINITY) || sum == 0.f;
        const float lse = empty ? INFINITY : __logf(sum) + mx;
        wsh[t] = empty ? 0.f : __expf(l0 - lse);
        wsh[t + 64] = empty ? 0.f : __expf(l1 - lse);
        if (cp.lse && t == 0) cp.lse[(int64_t)bidx * cp.lse_batch + (int64_t)head * cp.lse_head + pos] = lse;
    }
    __syncthreads();
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int sp = g + G * u;
        if (sp < ns) acc += wsh[sp] * x[u];
    }
    for (int s0 = g + G * NB; s0 < ns; s0 += G * NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int sp = s0 + G * u;
            x[u] = sp < ns ? *reinterpret_cast<const f32x4*>(oa + sp * sstride) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int sp = s0 + G * u;
            if (sp < ns) acc += wsh[sp] * x[u];
        }
    }
    red[g][c] = acc;
    __syncthreads();
    if (t < D4) {
        f32x4 o = red[0][t];
#pragma unroll
        for (int i = 1; i < G; ++i) o += red[i][t];
        T* orow = reinterpret_cast<T*>(cp.o) + (int64_t)bidx * cp.o_batch + (int64_t)pos * cp.o_row +
                  (int64_t)head * cp.o_head;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * t + i < cp.d) orow[4 * t + i] = (T)o[i];
    }
}

}  // namespace xfa

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

namespace xfa {

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
    if (FEAT) {
        if (p.cu_seqlens_q) { q_off = p.cu_seqlens_q[bidx]; sq = p.cu_seqlens_q[bidx + 1] - q_off; }
        if (p.cu_seqlens_k) { k_off = p.cu_seqlens_k[bidx]; sk = p.cu_seqlens_k[bidx + 1] - k_off; }
        if (p.seqused_k) sk = p.seqused_k[bidx];
    }
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
    const bool is_split = FEAT && p.num_splits > 1;
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
        const int qrow_off = (int)(((int64_t)pos * p.q_row + (int64_t)head * p.q_head) * 2);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int d0 = 16 * s + 8 * hh;
            const int off = (row_ok && d0 < p.d) ? qrow_off + d0 * 2 : kOOB;
            qf[s] = __builtin_bit_cast(V8, buf_load16(qr, off));
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
    auto load_tile = [&](int nb) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int n = nb * kBlockN + lrow0 + i * LROW_STEP;
            const bool ok = lc_ok && n < sk;
            if (paged) {
                const int nc = ok ? n : 0;
                const int pi = nc / p.page_size;
                const int pg = btab[pi];
                const int pr = nc - pi * p.page_size;
                const char* ka = kpool + ((int64_t)pg * p.k_batch + (int64_t)pr * p.k_row) * esz;
                const char* va = vpool + ((int64_t)pg * p.v_batch + (int64_t)pr * p.v_row) * esz;
                if (kv8) {
                    const uint2 kx = *reinterpret_cast<const uint2*>(ka);
                    const uint2 vx = *reinterpret_cast<const uint2*>(va);
                    kr[i] = ok ? fp8x8_to<T>(kx.x, kx.y, p.k_scale) : u32x4{0, 0, 0, 0};
                    vr[i] = ok ? fp8x8_to<T>(vx.x, vx.y, p.v_scale) : u32x4{0, 0, 0, 0};
                } else {
                    const u32x4 kx = *reinterpret_cast<const u32x4*>(ka);
                    const u32x4 vx = *reinterpret_cast<const u32x4*>(va);
                    kr[i] = ok ? kx : u32x4{0, 0, 0, 0};
                    vr[i] = ok ? vx : u32x4{0, 0, 0, 0};
                }
            } else if (kv8) {
                const u32x2 kx = buf_load8(krs, ok ? n * (int)p.k_row + lc * 8 : kOOB);
                const u32x2 vx = buf_load8(vrs, ok ? n * (int)p.v_row + lc * 8 : kOOB);
                kr[i] = fp8x8_to<T>(kx[0], kx[1], p.k_scale);
                vr[i] = fp8x8_to<T>(vx[0], vx[1], p.v_scale);
            } else {
                kr[i] = buf_load16(krs, ok ? n * (int)p.k_row * 2 + lc * 16 : kOOB);
                vr[i] = buf_load16(vrs, ok ? n * (int)p.v_row * 2 + lc * 16 : kOOB);
            }
        }
    };
    auto store_tile = [&](int buf) {
        char* ks = smem + buf * 2 * TILE;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int r = lrow0 + i * LROW_STEP;
            *reinterpret_cast<u32x4*>(ks + lds_off<HD>(r, lc)) = kr[i];
            *reinterpret_cast<u32x4*>(ks + TILE + lds_off<HD>(r, lc)) = vr[i];
        }
    };

    // Per-lane LDS read offsets (row-independent parts of the swizzle).
    int koff[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) koff[s] = lds_off<HD>(lr, 2 * s + hh);
    const int q4 = (lane & 15) >> 2;
    int voff[2][ND];
#pragma unroll
    for (int part = 0; part < 2; ++part) {
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
            const int r = 4 * hh + q4 + 8 * part;
            const int col = 32 * dt + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            voff[part][dt] = lds_off<HD>(r, col >> 3) + 8 * ((col >> 2) & 1);
        }
    }

    f32x16 acc_o[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) acc_o[dt] = f32x16{};
    float m_run = -INFINITY;
    float l_run = 0.f;

    if (nb_lo < nb_hi) {
        load_tile(nb_lo);
        store_tile(0);
    }
    // Retire every prologue load (the Q fragments) here: otherwise the loop-header merge of
    // the waitcnt scoreboard makes the first QK^T MFMA of EVERY iteration wait vmcnt(0), i.e.
    // drain the next tile's prefetch (vmcnt=0, expcnt=7, lgkmcnt=15).
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    if (p.prio_hi && __builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);
    int buf = 0;
    for (int nb = nb_lo; nb < nb_hi; ++nb) {
        const bool more = nb + 1 < nb_hi;
        if (more) load_tile(nb + 1);
        const char* ks = smem + buf * 2 * TILE;
        const char* vs = ks + TILE;
        const int n0 = nb * kBlockN;
        const bool active = wave_ok && n0 < w_lr_max && n0 + kBlockN > w_ll_min;
        if (active) {
            // ---- S^T = K Q^T : two 32-key tiles
            f32x16 st[2] = {f32x16{}, f32x16{}};
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const V8 a0 = *reinterpret_cast<const V8*>(ks + koff[s]);
                const V8 a1 = *reinterpret_cast<const V8*>(ks + 32 * HD * 2 + koff[s]);
                st[0] = DT<T>::mfma32(a0, qf[s], st[0]);
                st[1] = DT<T>::mfma32(a1, qf[s], st[1]);
            }
            // ---- score transforms + masking (only where a window edge crosses the tile)
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
            const bool need_mask = (n0 + kBlockN > w_lr_min) || (n0 < w_ll_max);
            if (need_mask) {
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int key = keyb + 32 * kt + (r & 3) + 8 * (r >> 2);
                        if (key >= my_lr || key < my_ll) st[kt][r] = -INFINITY;
                    }
            }
            // ---- online softmax (lane-local row + one half swap)
            float mx = st[0][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) mx = fmaxf(mx, st[0][r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[1][r]);
            mx = wave_max_halves(mx);
            const float m_new = fmaxf(m_run, mx);
            const float mref = (m_new == -INFINITY) ? 0.f : m_new * c;
            // Exact lazy rescale: only when some row of this wave raised its running max
            // (the O^T rescale is a 64-register VALU pass; after the first tiles it is rare).
            if (__any(m_new > m_run)) {
                const float alpha = fast_exp2(m_run * c - mref);
                l_run *= alpha;
#pragma unroll
                for (int dt = 0; dt < ND; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc_o[dt][r] *= alpha;
                m_run = m_new;
            }
            float rs[4] = {0.f, 0.f, 0.f, 0.f};   // 4 independent chains, not one 32-long
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float e = fast_exp2(fmaf(st[kt][r], c, -mref));
                    st[kt][r] = e;
                    rs[r & 3] += e;
                }
            l_run += (rs[0] + rs[1]) + (rs[2] + rs[3]);
            // ---- O^T += V^T P^T : P accumulator registers are the B operand as they stand
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {
                    V8 pb;
#pragma unroll
                    for (int j = 0; j < 8; ++j) pb[j] = (T)st[kt][8 * sp + j];
                    const int rbase = (32 * kt + 16 * sp) * HD * 2;
#pragma unroll
                    for (int dt = 0; dt < ND; ++dt) {
                        const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s16x4*)(vs + rbase + voff[0][dt]));
                        const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s16x4*)(vs + rbase + voff[1][dt]));
                        const s16x8 av = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
                        acc_o[dt] = DT<T>::mfma32(__builtin_bit_cast(V8, av), pb, acc_o[dt]);
                    }
                }
            }
        }
        if (more) store_tile(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }

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

// Grid: either one workgroup per item (grid = (b*hk, m_blocks, splits), heaviest causal row
// blocks dispatched first), or persistent (p.persistent: grid = (resident workgroups, 1,
// splits)), each workgroup walking items in a heaviest-first boustrophedon order so the
// causal work per workgroup balances, and one item's O-store tail overlaps the next item's
// prologue loads instead of a workgroup boundary.
template <int HD, typename T, int NW, bool MASK, bool FEAT>
__global__ void __launch_bounds__(NW * 64, 2) fmha_fwd_kernel(const FwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nbh = p.b * p.hk;
    const int g = gridDim.x;
    for (int k = 0;; ++k) {        // one call site: the item body is inlined once
        int bh, m_block;
        if (p.persistent) {
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
}

// Split-KV combine: lse = log sum_s exp(lse_s); O = sum_s exp(lse_s - lse) O_s
// (reference combine_attn_seqk_parallel, flash_fwd_kernel_hip.h:1322-1568; empty -> +inf).
// One wave per (b, h, pos) row.
template <int HD, typename T>
__global__ void __launch_bounds__(256) fmha_combine_kernel(const CombineParams cp) {
    const int lane = threadIdx.x & 63;
    const int64_t rid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t rows = (int64_t)cp.b * cp.h * cp.seqlen_q;
    if (rid >= rows) return;
    const int pos = (int)(rid % cp.seqlen_q);
    const int head = (int)((rid / cp.seqlen_q) % cp.h);
    const int bidx = (int)(rid / ((int64_t)cp.seqlen_q * cp.h));
    float mx = -INFINITY;
    for (int s = 0; s < cp.num_splits; ++s) mx = fmaxf(mx, cp.lseaccum[s * rows + rid]);
    float sum = 0.f;
    if (mx != -INFINITY)
        for (int s = 0; s < cp.num_splits; ++s) sum += __expf(cp.lseaccum[s * rows + rid] - mx);
    const bool empty = (mx == -INFINITY) || sum == 0.f;
    const float lse = empty ? INFINITY : __logf(sum) + mx;
    constexpr int PER = HD / 64;
    float acc[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) acc[i] = 0.f;
    if (!empty) {
        for (int s = 0; s < cp.num_splits; ++s) {
            const float w = __expf(cp.lseaccum[s * rows + rid] - lse);
            const float* oa = cp.oaccum + (s * rows + rid) * HD + lane * PER;
#pragma unroll
            for (int i = 0; i < PER; ++i) acc[i] = fmaf(w, oa[i], acc[i]);
        }
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

}  // namespace xfa

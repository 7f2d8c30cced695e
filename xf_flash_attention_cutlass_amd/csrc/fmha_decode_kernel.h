// fmha_decode_kernel.h — split-KV decode attention for gfx950 (CDNA4), HBM-bound.
//
// Replaces the decode use of the reference's split kernel (`fmha_page_kvcache_fwd`,
// csrc/paged_attn.cpp:442-568 -> compute_attn_1rowblock_splitkv, flash_fwd_kernel_hip.h:585-1283
// with num_splits > 1, + combine_attn_seqk_parallel :1322-1568) for the case the whole GQA group
// of query rows (seqlen_q * H/Hk <= 32) fits one 32-row MFMA tile.  Decode reads every K/V
// byte exactly once, so the design goal is bytes in flight, not MFMA rate:
//
//  * every wave is its own split: a 4-wave workgroup owns one (batch, kv head) and 4 key
//    ranges; no barrier, no workgroup-level LDS sharing;
//  * K and V are loaded coalesced (consecutive lanes read consecutive 16-byte chunks of a
//    row), dequantised, and written to a wave-private 32-key LDS image (the swizzled image of
//    fmha_common.h), from which K is read as the A operand of S^T = K Q^T and V transposed
//    (ds_read_b64_tr_b16) as the A operand of O^T += V^T P^T — a lane-per-key register
//    layout would make every load instruction touch 32 rows with one 16-byte piece each;
//  * fp8 (OCP e4m3fn) K/V are dequantised with v_cvt_scalef32_pk_{bf16,f16}_fp8 (exact for
//    e4m3 -> bf16/f16); the per-tensor scales are applied to S (k_scale) and O (v_scale) in
//    fp32, never to the stored operands;
//  * a ring of raw K/V registers keeps the next tiles' loads in flight across the compute of
//    the current tile (two tiles for fp8, one for 16-bit caches): a slot is refilled with the
//    tile RING ahead as soon as its raw bytes are converted;
//  * partial (O, LSE) per wave go to the split scratch; fmha_combine_kernel merges them.
#pragma once

#include "fmha_common.h"

namespace xfa {

constexpr int kDecKeys = 32;        // keys per tile (one 32x32 MFMA block of S^T)
constexpr int kDecWaves = 4;        // waves (= splits) per workgroup

template <typename T> struct FP8Cvt;
template <> struct FP8Cvt<__bf16> {
    // 4 fp8 in one dword -> 4 bf16 in two dwords
    static __device__ __forceinline__ u32x2 cvt4(unsigned w) {
        const auto lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.0f, false);
        const auto hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.0f, true);
        return u32x2{__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi)};
    }
};
template <> struct FP8Cvt<_Float16> {
    static __device__ __forceinline__ u32x2 cvt4(unsigned w) {
        const auto lo = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 1.0f, false);
        const auto hi = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 1.0f, true);
        return u32x2{__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi)};
    }
};

template <int HD, typename T, bool KV8>
__global__ void __launch_bounds__(kDecWaves * 64, 2) fmha_decode_kernel(const FwdParams p) {
    using V8 = typename DT<T>::v8;
    constexpr int NS = HD / 16;                  // k-steps of S^T = K Q^T
    constexpr int ND = HD / 32;                  // 32-wide d tiles of O^T
    constexpr int ESZ = KV8 ? 1 : 2;
    constexpr int CPR = HD * ESZ / 16;           // 16-byte chunks per K (V) row
    constexpr int RPI = 64 / CPR;                // rows per load instruction
    constexpr int NLD = kDecKeys / RPI;          // load instructions per lane per K (V) tile
    constexpr int RING = KV8 ? 2 : 1;            // tiles in flight beyond the current one
    constexpr int SLICE = kDecKeys * HD * 2;     // LDS bytes of one wave's K (or V) image
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31;
    const int hh = lane >> 5;
    const int bh = blockIdx.x;
    const int bidx = bh / p.hk;
    const int hk_i = bh - bidx * p.hk;
    const int split = blockIdx.y * kDecWaves + wave;
    char* vsl = smem + wave * 2 * SLICE;         // this wave's V image; K image follows

    const int sq = p.seqlen_q;
    const int sk = p.seqused_k ? p.seqused_k[bidx] : p.seqlen_k;
    const int G = p.group;
    const int rows = sq * G;
    const int diag = sk - sq;
    auto lim_r = [&](int pos) { return p.wr >= 0 ? min(sk, pos + diag + p.wr + 1) : sk; };
    auto lim_l = [&](int pos) { return p.wl >= 0 ? max(0, pos + diag - p.wl) : 0; };

    // this lane's query row (MFMA column)
    const bool row_ok = lr < rows;
    const int pos = row_ok ? lr / G : 0;
    const int head = hk_i * G + (row_ok ? lr - pos * G : 0);
    const int my_lr = lim_r(pos), my_ll = lim_l(pos);
    float alibi_w = 0.f;
    if (p.alibi) alibi_w = p.alibi[bidx * p.alibi_bstride + head] * p.alibi_mul;
    const float c = p.scale_log2;

    // key tiles of this split (the union of every row's window, cut into num_splits ranges)
    const int k_lo = lim_l(0), k_hi = lim_r(rows > 0 ? (rows - 1) / G : 0);
    const int t_first = k_lo / kDecKeys;
    const int t_end = k_hi > k_lo ? (k_hi + kDecKeys - 1) / kDecKeys : t_first;
    const int per = (t_end - t_first + p.num_splits - 1) / p.num_splits;
    const int t_lo = min(t_end, t_first + split * per);
    const int t_hi = min(t_end, t_lo + per);

    // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[row][16s + 8hh .. +7]
    V8 qf[NS];
    {
        const T* qrow = reinterpret_cast<const T*>(p.q) + (int64_t)bidx * p.q_batch +
                        (int64_t)pos * p.q_row + (int64_t)head * p.q_head + 8 * hh;
#pragma unroll
        for (int s = 0; s < NS; ++s)
            qf[s] = row_ok ? *reinterpret_cast<const V8*>(qrow + 16 * s) : V8{};
    }

    // ---- K/V loads, coalesced: instruction i, lane l -> tile row RPI*i + l / CPR, 16-byte
    // chunk l % CPR of that row (consecutive lanes read consecutive bytes of one row)
    const bool paged = p.block_table != nullptr;
    const int lrow = lane / CPR, lch = lane % CPR;
    const char* kbase = reinterpret_cast<const char*>(p.k) + (int64_t)hk_i * p.k_head * ESZ + 16 * lch;
    const char* vbase = reinterpret_cast<const char*>(p.v) + (int64_t)hk_i * p.v_head * ESZ + 16 * lch;
    if (!paged) {
        kbase += (int64_t)bidx * p.k_batch * ESZ;
        vbase += (int64_t)bidx * p.v_batch * ESZ;
    }
    // Page-table entries are wave-uniform per (tile, page): a 32-key tile spans at most two
    // pages when page_size % 16 == 0 (the host guarantees it), so they are scalar loads through
    // the constant address space (lgkm-counted: they never make the vector-load ring drain),
    // fetched one tile early.
    typedef __attribute__((address_space(4))) const int cint;
    cint* btab = paged ? (cint*)(p.block_table + (int64_t)bidx * p.bt_stride) : nullptr;
    int pg_next[2] = {0, 0};
    auto fetch_pages = [&](const int t, int (&pg)[2]) {
        if (!paged) return;
        const int last = (sk - 1) / p.page_size;
        const int pi0 = __builtin_amdgcn_readfirstlane(min((t * kDecKeys) / p.page_size, last));
        pg[0] = btab[pi0];
        pg[1] = btab[min(pi0 + 1, last)];
    };

    u32x4 kraw[RING][NLD], vraw[RING][NLD];
    auto issue = [&](const int t, const int (&pg)[2], u32x4 (&kr)[NLD], u32x4 (&vr)[NLD]) {
        int64_t ko[NLD], vo[NLD];
        if (paged) {
            const int pi0 = (t * kDecKeys) / p.page_size;
#pragma unroll
            for (int i = 0; i < NLD; ++i) {
                const int n = min(t * kDecKeys + RPI * i + lrow, sk - 1);   // clamped rows
                const int pi = n / p.page_size;
                const int pgl = pi == pi0 ? pg[0] : pg[1];
                const int pr = n - pi * p.page_size;
                ko[i] = ((int64_t)pgl * p.k_batch + (int64_t)pr * p.k_row) * ESZ;
                vo[i] = ((int64_t)pgl * p.v_batch + (int64_t)pr * p.v_row) * ESZ;
            }
        } else {
#pragma unroll
            for (int i = 0; i < NLD; ++i) {
                const int n = min(t * kDecKeys + RPI * i + lrow, sk - 1);
                ko[i] = (int64_t)n * p.k_row * ESZ;
                vo[i] = (int64_t)n * p.v_row * ESZ;
            }
        }
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            kr[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(kbase + ko[i]));
            vr[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(vbase + vo[i]));
        }
    };

    // ---- wave-private LDS images (swizzled, fmha_common.h): K rows read as the A operand of
    // S^T (ds_read_b128), V read transposed as the A operand of O^T (ds_read_b64_tr_b16)
    char* ksl = vsl + SLICE;
    // write offsets of this lane's 8-element chunk(s) (fp8: a 16-byte load is two chunks)
    int kw[NLD][3 - ESZ];
#pragma unroll
    for (int i = 0; i < NLD; ++i)
#pragma unroll
        for (int h2 = 0; h2 < 3 - ESZ; ++h2) kw[i][h2] = lds_off<HD>(RPI * i + lrow, (3 - ESZ) * lch + h2);
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

    // prologue: RING tiles in flight, pages of the next one fetched
    if (t_lo < t_hi) {
#pragma unroll
        for (int r = 0; r < RING; ++r) {
            int pg[2];
            fetch_pages(min(t_lo + r, t_hi - 1), pg);
            issue(min(t_lo + r, t_hi - 1), pg, kraw[r], vraw[r]);
            __builtin_amdgcn_sched_barrier(0);    // slot order = issue order (waitcnt merge)
        }
        fetch_pages(min(t_lo + RING, t_hi - 1), pg_next);
    }
    // Retire the Q loads (issued before the ring) explicitly: otherwise the loop-header merge
    // of the waitcnt scoreboard makes the first tile of every iteration wait vmcnt(0).
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * NLD * RING));

    // one tile; `slot` is compile-time (the ring is unrolled)
    auto tile = [&](auto SLOT, const int t) {
        constexpr int slot = decltype(SLOT)::value;
        // raw chunks -> T -> LDS images (fp8: 16 values = two 8-element chunks)
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            if constexpr (KV8) {
                const u32x2 a = FP8Cvt<T>::cvt4(kraw[slot][i][0]), b = FP8Cvt<T>::cvt4(kraw[slot][i][1]);
                const u32x2 c2 = FP8Cvt<T>::cvt4(kraw[slot][i][2]), d = FP8Cvt<T>::cvt4(kraw[slot][i][3]);
                *reinterpret_cast<u32x4*>(ksl + kw[i][0]) = u32x4{a[0], a[1], b[0], b[1]};
                *reinterpret_cast<u32x4*>(ksl + kw[i][1]) = u32x4{c2[0], c2[1], d[0], d[1]};
                const u32x2 e = FP8Cvt<T>::cvt4(vraw[slot][i][0]), f = FP8Cvt<T>::cvt4(vraw[slot][i][1]);
                const u32x2 g = FP8Cvt<T>::cvt4(vraw[slot][i][2]), h = FP8Cvt<T>::cvt4(vraw[slot][i][3]);
                *reinterpret_cast<u32x4*>(vsl + kw[i][0]) = u32x4{e[0], e[1], f[0], f[1]};
                *reinterpret_cast<u32x4*>(vsl + kw[i][1]) = u32x4{g[0], g[1], h[0], h[1]};
            } else {
                *reinterpret_cast<u32x4*>(ksl + kw[i][0]) = kraw[slot][i];
                *reinterpret_cast<u32x4*>(vsl + kw[i][0]) = vraw[slot][i];
            }
        }
        // Pin the LDS writes before the refill: if the refill is hoisted above them the slot's
        // registers are renamed and the loop copies them back at its end - which waits for the
        // refill, i.e. drains the ring every tile.
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // keep the ring full: the tile RING ahead goes into the slot just written out
        // (unconditional, clamped to the last tile: a conditional refill would make the
        // compiler's loop-header waitcnt merge drain the whole ring every tile)
        issue(min(t + RING, t_hi - 1), pg_next, kraw[slot], vraw[slot]);
        fetch_pages(min(t + RING + 1, t_hi - 1), pg_next);
        V8 kf[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) kf[s] = *reinterpret_cast<const V8*>(ksl + koff[s]);
        // S^T = K Q^T
        f32x16 st{};
#pragma unroll
        for (int s = 0; s < NS; ++s) st = DT<T>::mfma32(kf[s], qf[s], st);
        // scale / transforms / mask
        const int keyb = t * kDecKeys + 4 * hh;
        const bool edge = (t + 1) * kDecKeys > min(sk, my_lr) || t * kDecKeys < my_ll;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float x = st[r];
            if (KV8) x *= p.k_scale;
            if (p.softcap_pre > 0.f) x = fast_tanh(x * p.softcap_pre);
            const int key = keyb + (r & 3) + 8 * (r >> 2);
            if (p.alibi) x -= alibi_w * (float)abs(pos + diag - key);
            if (edge && (key >= my_lr || key < my_ll)) x = -INFINITY;
            st[r] = x;
        }
        float mx = st[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, st[r]);
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
        V8 pb[2];
        float rs = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float e = fast_exp2(fmaf(st[r], c, -mref));
            rs += e;
            pb[r >> 3][r & 7] = (T)e;
        }
        l_run += rs;
        // O^T += V^T P^T (keys permuted as in fmha_fwd_kernel.h)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
            for (int dt = 0; dt < ND; ++dt) {
                const char* b = vsl + 16 * sp * HD * 2;
                const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + voff[0][dt]));
                const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + voff[1][dt]));
                const s16x8 av = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
                acc_o[dt] = DT<T>::mfma32(__builtin_bit_cast(V8, av), pb[sp], acc_o[dt]);
            }
    };

    int t = t_lo;
    if constexpr (RING == 2) {
        // whole pairs in a loop without a mid-body exit (keeps the waitcnt merge exact), then
        // the odd last tile
        for (; t + 1 < t_hi; t += 2) {
            tile(std::integral_constant<int, 0>{}, t);
            tile(std::integral_constant<int, 1>{}, t + 1);
        }
        if (t < t_hi) tile(std::integral_constant<int, 0>{}, t);
    } else {
        for (; t < t_hi; ++t) tile(std::integral_constant<int, 0>{}, t);
    }

    // ---- split partial: O (fp32, normalised, v_scale applied) + LSE; empty -> O = 0, -inf
    const float l_full = wave_sum_halves(l_run);
    const bool empty = (l_full == 0.f) || (l_full != l_full);
    const float inv = empty ? 0.f : (KV8 ? p.v_scale : 1.f) / l_full;
    if (!row_ok) return;
    const int64_t rid = (((int64_t)split * p.b + bidx) * p.h + head) * sq + pos;
    float* oa = p.oaccum + rid * HD;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int d = 32 * dt + 8 * g + 4 * hh;
            *reinterpret_cast<f32x4*>(oa + d) = f32x4{acc_o[dt][4 * g] * inv, acc_o[dt][4 * g + 1] * inv,
                                                      acc_o[dt][4 * g + 2] * inv, acc_o[dt][4 * g + 3] * inv};
        }
    if (hh == 0) p.lseaccum[rid] = empty ? -INFINITY : (m_run * c + __log2f(l_full)) * kLn2;
}

}  // namespace xfa

// fmha_decode_kernel.h — split-KV decode attention for gfx950 (CDNA4), HBM-bound.
//
// Replaces the decode use of the reference's split kernel (`fmha_page_kvcache_fwd`,
// csrc/paged_attn.cpp:442-568 -> compute_attn_1rowblock_splitkv, flash_fwd_kernel_hip.h:585-1283
// with num_splits > 1, + combine_attn_seqk_parallel :1322-1568) for the case the whole GQA group
// of query rows (seqlen_q * H/Hk <= 32) fits one 32-row MFMA tile.  Decode reads every K/V
// byte exactly once, so the design goal is bytes in flight, not MFMA rate:
//
//  * every wave is its own split, no barrier, no workgroup-level LDS sharing; the waves of a
//    workgroup are 4 (or 8) kv heads of one (batch, key range) — their rows sit side by side in
//    every cache row, so a workgroup's loads cover contiguous 512 B (1 KiB) runs of each row
//    (dec_hmaj; +5 % on C5 over 4 key ranges of one kv head, whose 128-byte fp8 rows are 1 KiB
//    apart);
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
//  * partial (O, LSE) per wave go to the split scratch; fmha_combine_kernel merges them;
//  * MR = 16 (GQA groups of <= 16 query rows, the common decode shape): S^T and O^T on
//    v_mfma_f32_16x16x32 — half the MFMA cycles and half the softmax lanes of the 32-row tile,
//    and the freed registers deepen the load ring (3 fp8 tiles in flight instead of 2).
//    Lane l holds query row l % 16 and, of each 16-key block, keys 4 (l / 16) .. +3; the two
//    blocks' P values are directly the B operand of the PV product with its k index permuted
//    to key(8g + i) = i < 4 ? 4g + i : 16 + 4g + (i - 4), the same permutation applied to V^T.
#pragma once

#include "fmha_common.h"

namespace xfa {

// Cache policy of the K/V stream loads (buffer aux bits): 2 = `nt`, the non-temporal hint.
// Decode reads every cache byte exactly once, so the lines need not stay in L2 / the
// Infinity Cache: C5 0.1034 -> 0.0918 ms (5.19 -> 5.85 TB/s, same box, bit-identical); `sc0`
// (1) no change.  (The forward keeps the default policy: its K/V tiles are re-read by every
// row block of a head.)
#ifndef XFA_DEC_CPOL
#define XFA_DEC_CPOL 2
#endif

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

template <typename T> __device__ __forceinline__ f32x4 dec_mfma16(const typename DT<T>::v8& a,
                                                                const typename DT<T>::v8& b, const f32x4& c);
template <> __device__ __forceinline__ f32x4 dec_mfma16<__bf16>(const bf16x8& a, const bf16x8& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <> __device__ __forceinline__ f32x4 dec_mfma16<_Float16>(const f16x8& a, const f16x8& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// reductions over the four 16-lane groups that hold one query row (MR = 16)
__device__ __forceinline__ float quad_max16(float x) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float quad_sum16(float x) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Key tiles of sequence `b` that some query row can see (the union of the rows' windows):
// [t_first, t_end) in kDecKeys-key tiles; the decode kernel cuts exactly this range into splits.
__device__ __forceinline__ int2 dec_tile_range(const FwdParams& p, const int b) {
    const int lp = p.leftpad_k ? p.leftpad_k[b] : 0;
    const int sk = (p.seqused_k ? p.seqused_k[b] : p.seqlen_k) - lp;
    const int rows = p.seqlen_q * p.group;
    const int diag = sk - p.seqlen_q;
    const int last = rows > 0 ? (rows - 1) / p.group : 0;
    const int k_lo = p.wl >= 0 ? max(0, diag - p.wl) : 0;
    const int k_hi = p.wr >= 0 ? min(sk, last + diag + p.wr + 1) : sk;
    const int t_first = k_lo / kDecKeys;
    const int t_end = k_hi > k_lo ? (k_hi + kDecKeys - 1) / kDecKeys : t_first;
    return int2{t_first, t_end};
}

// Balanced split allocation over ragged caches (`dec_bal`): the p.dec_slots split slots of one
// kv-head group are shared by the sequences in proportion to their key tiles, at least one each
// and at most p.dec_cap (the scratch's split extent): sequence b owns slots
// [S_b, S_b + n_b) with n_b = 1 + floor(E (C_b + T_b) / T) - floor(E C_b / T), E = slots - B,
// C_b = the tiles of the sequences before b, T = all tiles.  Equal lengths give n_b =
// slots / B, i.e. the per-sequence split of the uniform launch (same ranges, same result).
// Lane b computes sequence b's share (b < B <= 64, one vector load of the lengths), the
// prefix sums run across the wave.  Slot f -> (sequence, split, n_b); false for a slot past the
// last sequence's.
__device__ __forceinline__ unsigned wave_incl_scan(unsigned x, const int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}
__device__ __forceinline__ bool dec_slot(const FwdParams& p, const int f, const int lane,
                                         int& bidx, int& split, int& nsb) {
    const bool own = lane < p.b;
    unsigned tb = 0;
    if (own) {
        const int2 r = dec_tile_range(p, lane);
        tb = (unsigned)(r.y - r.x);
    }
    const unsigned incl = wave_incl_scan(tb, lane);
    const uint64_t total = __shfl(incl, 63);
    const uint64_t extra = (uint64_t)(p.dec_slots - p.b);
    int n = 0;
    if (own) {
        n = 1 + (total > 0 ? (int)(extra * incl / total - extra * (incl - tb) / total) : 0);
        n = min(n, p.dec_cap);
    }
    const unsigned send = wave_incl_scan((unsigned)n, lane);
    const uint64_t hit = __ballot(own && (unsigned)f < send);
    if (!hit) return false;
    bidx = __builtin_ctzll(hit);
    nsb = __shfl(n, bidx);
    split = f - (int)(__shfl(send, bidx) - (unsigned)nsb);
    return true;
}

// Decode image for D = 128 with the 16-row tile (dec_mr 16).  Lane l reads K row l % 16 at
// chunk 4s + l / 16 (ds_read_b128: lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) and
// V^T rows 4 (l / 16) + (l % 16) / 4 of its 32-lane half (ds_read_b64_tr_b16); the forward's
// swz<128> (built for the 32-row tile's lane map) put two lanes of every such group on one bank —
// half of the decode's LDS cycles were conflicts (r03b PMC).  This map is conflict-free for both:
// a K group's 16 (row, chunk) pairs need f(rows 4..11) closed under ^1, a V half's 8 rows need
// distinct f(row) >> 1 — rows 0-7 -> 2r, rows 8-11 -> the odd partners of rows 4-7, rows 12-15 ->
// those of rows 0-3 (period 16 rows).  Chunks 8-15 also swap within their ^1 pairs (c ^ c[3]): a
// fp8 dequant store writes the 8 even (or odd) chunks of one row from an 8-lane group, which the
// 32-bank store path saw as 4 slots twice; now 8 (uniform per read instruction, so the reads keep
// their property).  Bank-checked for every instruction of the loop in tools/decode_banks.py.
__device__ __forceinline__ int dswz16(int row) {
    const int r = row & 15;
    return r < 8 ? 2 * r : (r < 12 ? 2 * r - 7 : 2 * r - 23);
}
template <int HD, int MR> __device__ __forceinline__ int dec_off(int row, int chunk) {
    if constexpr (HD == 128 && MR == 16) return row * (HD * 2) + ((chunk ^ ((chunk >> 3) & 1) ^ dswz16(row)) << 4);
    else return lds_off<HD>(row, chunk);
}

template <int HD, typename T, bool KV8, int MR, int NWV = kDecWaves>
__global__ void __launch_bounds__(NWV * 64, 2) fmha_decode_kernel(const FwdParams p) {
    using V8 = typename DT<T>::v8;
    static_assert(MR == 16 || MR == 32, "MFMA rows");
    constexpr int NS = MR == 32 ? HD / 16 : HD / 32;   // k-steps of S^T = K Q^T
    constexpr int ND = HD / MR;                  // MR-wide d tiles of O^T
    constexpr int NA = MR == 32 ? 16 : 4;        // accumulator registers per MR x MR tile
    typedef float __attribute__((ext_vector_type(NA))) accv;
    constexpr int ESZ = KV8 ? 1 : 2;
    constexpr int CPR = HD * ESZ / 16;           // 16-byte chunks per K (V) row
    constexpr int RPI = 64 / CPR;                // rows per load instruction
    constexpr int NLD = kDecKeys / RPI;          // load instructions per lane per K (V) tile
    // tiles in flight beyond the current one (bounded by the 256-VGPR budget of two waves
    // per SIMD; the 16-row tile frees the registers for one more fp8 tile)
    constexpr int RING = KV8 ? (MR == 16 ? 3 : 2) : 1;
    constexpr int SLICE = kDecKeys * HD * 2;     // LDS bytes of one wave's K (or V) image
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & (MR - 1);               // query row (MFMA column) of this lane
    const int hh = lane / MR;                     // key sub-block (0..64/MR-1) of this lane
    // wave -> (batch, kv head, split): 4 splits of one kv head, or (dec_hmaj) 4 kv heads of one
    // split, whose rows sit side by side in each cache row (HD * ESZ bytes apart)
    int bidx, hk_i, split, nsplit = p.num_splits;
    if (p.dec_bal) {
        // the head-major grid; slot f = x-batch * num_splits + y (for equal lengths exactly the
        // head-major launch's (batch, split), dispatched in the same order) -> (sequence, split)
        const int g4 = p.hk / NWV;
        const int xb = blockIdx.x / g4;
        hk_i = (blockIdx.x - xb * g4) * NWV + wave;
        if (!dec_slot(p, xb * p.num_splits + blockIdx.y, lane, bidx, split, nsplit)) return;
        bidx = __builtin_amdgcn_readfirstlane(bidx);
        split = __builtin_amdgcn_readfirstlane(split);
        nsplit = __builtin_amdgcn_readfirstlane(nsplit);
        if (split == 0 && hk_i == 0 && lane == 0) p.dec_ns[bidx] = nsplit;  // for the combine
    } else if (p.dec_hmaj) {
        const int g4 = p.hk / NWV;
        bidx = blockIdx.x / g4;
        hk_i = (blockIdx.x - bidx * g4) * NWV + wave;
        split = blockIdx.y;
    } else {
        bidx = blockIdx.x / p.hk;
        hk_i = blockIdx.x - bidx * p.hk;
        split = blockIdx.y * kDecWaves + wave;
    }
    char* vsl = smem + wave * 2 * SLICE;         // this wave's V image; K image follows

    const int sq = p.seqlen_q;
    // cache_leftpad: the sequence is cache rows [lp, seqused_k) (paged addressing only; the
    // host allows it for one-page-per-sequence caches, where no load group can straddle a page)
    const int lp = __builtin_amdgcn_readfirstlane(p.leftpad_k ? p.leftpad_k[bidx] : 0);
    const int sk = __builtin_amdgcn_readfirstlane(p.seqused_k ? p.seqused_k[bidx] : p.seqlen_k) - lp;
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
    const int per = (t_end - t_first + nsplit - 1) / nsplit;
    const int t_lo = min(t_end, t_first + split * per);
    const int t_hi = min(t_end, t_lo + per);

    // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[row][KS s + 8hh .. +7]
    // (KS = the k depth of one MFMA: 16 for 32x32x16, 32 for 16x16x32)
    constexpr int KS = MR == 32 ? 16 : 32;
    V8 qf[NS];
    {
        const T* qrow = reinterpret_cast<const T*>(p.q) + (int64_t)bidx * p.q_batch +
                        (int64_t)pos * p.q_row + (int64_t)head * p.q_head + 8 * hh;
#pragma unroll
        for (int s = 0; s < NS; ++s)
            qf[s] = row_ok ? *reinterpret_cast<const V8*>(qrow + KS * s) : V8{};
    }

    // ---- K/V loads, coalesced: instruction i, lane l -> tile row RPI*i + l / CPR, 16-byte
    // chunk l % CPR of that row (consecutive lanes read consecutive bytes of one row).
    // Addressing is scalar: one load instruction covers RPI <= 8 rows, which never straddle a
    // page (pages are multiples of 16 rows, host-checked), so its page and row are wave-uniform
    // and go into a buffer descriptor and soffset; the per-lane part (row in the group, chunk)
    // is a loop-invariant voffset.  (Per-lane 64-bit paged address arithmetic — a division by
    // the page size per row — was the decode kernel's largest instruction cost.)
    const bool paged = p.block_table != nullptr;
    const int lrow = lane / CPR, lch = lane % CPR;
    const int lane_k = lrow * (int)p.k_row * ESZ + 16 * lch;
    const int lane_v = lrow * (int)p.v_row * ESZ + 16 * lch;
    const char* kpool = reinterpret_cast<const char*>(p.k) + (int64_t)hk_i * p.k_head * ESZ;
    const char* vpool = reinterpret_cast<const char*>(p.v) + (int64_t)hk_i * p.v_head * ESZ;
    if (!paged) {
        kpool += (int64_t)bidx * p.k_batch * ESZ;
        vpool += (int64_t)bidx * p.v_batch * ESZ;
    }
    kpool = uniform_ptr(kpool);
    vpool = uniform_ptr(vpool);
    const int krow_b = (int)p.k_row * ESZ, vrow_b = (int)p.v_row * ESZ;
    // Page-table entries are wave-uniform per (tile, page): a 32-key tile spans at most two
    // pages, so they are scalar loads through the constant address space (lgkm-counted: they
    // never make the vector-load ring drain), fetched one tile early, together with the row of
    // the tile start inside its first page.
    typedef __attribute__((address_space(4))) const int cint;
    cint* btab = paged ? (cint*)(p.block_table + (int64_t)bidx * p.bt_stride) : nullptr;
    int pg_next[3] = {0, 0, 0};
    auto fetch_pages = [&](const int t, int (&pg)[3]) __attribute__((always_inline)) {
        if (!paged) return;
        const int last = (sk + lp - 1) / p.page_size;
        const int pi0 = __builtin_amdgcn_readfirstlane(min((t * kDecKeys + lp) / p.page_size, last));
        pg[0] = btab[pi0];
        pg[1] = btab[min(pi0 + 1, last)];
        pg[2] = t * kDecKeys + lp - pi0 * p.page_size;    // may exceed the page past the last row
    };
    const uint32_t page_k = (uint32_t)(p.page_size * krow_b), page_v = (uint32_t)(p.page_size * vrow_b);
    const __amdgpu_buffer_rsrc_t kseq_rs =
        make_rsrc(kpool, paged ? 0u : (uint32_t)min((int64_t)sk * krow_b, (int64_t)0xFFFFFFFF));
    const __amdgpu_buffer_rsrc_t vseq_rs =
        make_rsrc(vpool, paged ? 0u : (uint32_t)min((int64_t)sk * vrow_b, (int64_t)0xFFFFFFFF));

    u32x4 kraw[RING][NLD], vraw[RING][NLD];
    auto issue = [&](const int t, const int (&pg)[3], u32x4 (&kr)[NLD], u32x4 (&vr)[NLD]) __attribute__((always_inline)) {
        if (paged) {
            // past the last key the page index is clamped, so the rows of a group that wraps
            // there re-read rows of the last page: keys >= seqlen, masked in registers
#pragma unroll
            for (int i = 0; i < NLD; ++i) {
                // (readfirstlane: the divergence analysis loses the uniformity of the page
                // entries, and a descriptor it believes divergent becomes a waterfall loop)
                int x = __builtin_amdgcn_readfirstlane(pg[2] + RPI * i);
                const bool nxt = x >= p.page_size;
                const int page = __builtin_amdgcn_readfirstlane(nxt ? pg[1] : pg[0]);
                x = nxt ? x - p.page_size : x;
                // the page base through readfirstlane: computed with a VALU 64-bit multiply-add,
                // a base left in VGPRs made every load a (single-trip) waterfall loop
                const __amdgpu_buffer_rsrc_t krs = make_rsrc(uniform_ptr(kpool + (int64_t)page * p.k_batch * ESZ), page_k);
                const __amdgpu_buffer_rsrc_t vrs = make_rsrc(uniform_ptr(vpool + (int64_t)page * p.v_batch * ESZ), page_v);
                kr[i] = __builtin_amdgcn_raw_buffer_load_b128(krs, lane_k, x * krow_b, XFA_DEC_CPOL);
                vr[i] = __builtin_amdgcn_raw_buffer_load_b128(vrs, lane_v, x * vrow_b, XFA_DEC_CPOL);
            }
        } else {
            // rows >= sk fall outside the sequence descriptor and read as zeros
#pragma unroll
            for (int i = 0; i < NLD; ++i) {
                const int n = t * kDecKeys + RPI * i;
                kr[i] = __builtin_amdgcn_raw_buffer_load_b128(kseq_rs, lane_k, n * krow_b, XFA_DEC_CPOL);
                vr[i] = __builtin_amdgcn_raw_buffer_load_b128(vseq_rs, lane_v, n * vrow_b, XFA_DEC_CPOL);
            }
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
        for (int h2 = 0; h2 < 3 - ESZ; ++h2) kw[i][h2] = dec_off<HD, MR>(RPI * i + lrow, (3 - ESZ) * lch + h2);
    // K operand (A of S^T) of k-step s: row lr (key), 16-byte chunk s KS/8 + hh; the second
    // 16-key block (MR = 16) is 16 rows on, same swizzle (the swizzle has period 16)
    int koff[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) koff[s] = dec_off<HD, MR>(lr, (KS / 8) * s + hh);
    // V^T operand (A of O^T) through ds_read_b64_tr_b16: a 16-lane group reads a 4-key x
    // 16-column block and each lane receives its column's 4 keys
    const int q4 = (lane & 15) >> 2;
    int voff[2][ND];
#pragma unroll
    for (int part = 0; part < 2; ++part)
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
            if constexpr (MR == 32) {
                const int r = 4 * hh + q4 + 8 * part;
                const int col = 32 * dt + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
                voff[part][dt] = dec_off<HD, MR>(r, col >> 3) + 8 * ((col >> 2) & 1);
            } else {
                const int r = 4 * hh + q4 + 16 * part;  // keys 4g.. and 16+4g.. of the tile
                const int col = 16 * dt + 4 * (lane & 3);
                voff[part][dt] = dec_off<HD, MR>(r, col >> 3) + 8 * ((col >> 2) & 1);
            }
        }

    accv acc_o[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) acc_o[dt] = accv{};
    float m_run = -INFINITY, l_run = 0.f;

    // prologue: RING tiles in flight, pages of the next one fetched
    if (t_lo < t_hi) {
#pragma unroll
        for (int r = 0; r < RING; ++r) {
            int pg[3] = {0, 0, 0};
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
    auto tile = [&](auto SLOT, const int t) __attribute__((always_inline)) {
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
        // S^T = K Q^T: MR = 32 one 32x32 block of 32 keys; MR = 16 two 16x16 blocks
        constexpr int NKB = MR == 32 ? 1 : 2;
        accv st[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            V8 kf[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) kf[s] = *reinterpret_cast<const V8*>(ksl + koff[s] + kb * 16 * HD * 2);
            st[kb] = accv{};
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                if constexpr (MR == 32) st[kb] = DT<T>::mfma32(kf[s], qf[s], st[kb]);
                else st[kb] = dec_mfma16<T>(kf[s], qf[s], st[kb]);
            }
        }
        // scale / transforms / mask; element (kb, r) is key t*32 + keyof(kb, r)
        auto keyof = [&](const int kb, const int r) {
            return MR == 32 ? 4 * hh + (r & 3) + 8 * (r >> 2) : 16 * kb + 4 * hh + r;
        };
        const int keyb = t * kDecKeys;
        // Softcap / ALiBi and the window edge behind wave-uniform branches: written as per-score
        // conditions, the compiler if-converted them and ran tanh (exp + rcp) and the ALiBi
        // distance on every score of every tile
        const bool edge = (t + 1) * kDecKeys > min(sk, my_lr) || t * kDecKeys < my_ll;
        if (KV8) {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int r = 0; r < NA; ++r) st[kb][r] *= p.k_scale;
        }
        if (p.softcap_pre > 0.f || p.alibi) {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int r = 0; r < NA; ++r) {
                    float x = st[kb][r];
                    if (p.softcap_pre > 0.f) x = fast_tanh(x * p.softcap_pre);
                    if (p.alibi) x -= alibi_w * (float)abs(pos + diag - (keyb + keyof(kb, r)));
                    st[kb][r] = x;
                }
        }
        if (__builtin_amdgcn_ballot_w64(edge)) {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int r = 0; r < NA; ++r) {
                    const int key = keyb + keyof(kb, r);
                    if (edge && (key >= my_lr || key < my_ll)) st[kb][r] = -INFINITY;
                }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int r = 0; r < NA; ++r) mx = fmaxf(mx, st[kb][r]);
        mx = MR == 32 ? wave_max_halves(mx) : quad_max16(mx);
        const float m_new = fmaxf(m_run, mx);
        const float mref = (m_new == -INFINITY) ? 0.f : m_new * c;
        if (__any(m_new > m_run)) {
            const float alpha = fast_exp2(m_run * c - mref);
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < ND; ++dt)
#pragma unroll
                for (int r = 0; r < NA; ++r) acc_o[dt][r] *= alpha;
            m_run = m_new;
        }
        // P -> T: the B operand of the PV product (keys permuted as in the header comment)
        constexpr int NPB = MR == 32 ? 2 : 1;
        V8 pb[NPB];
        float rs = 0.f;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int r = 0; r < NA; ++r) {
                const float e = fast_exp2(fmaf(st[kb][r], c, -mref));
                rs += e;
                const int i = kb * NA + r;
                pb[i >> 3][i & 7] = (T)e;
            }
        l_run += rs;
        // O^T += V^T P^T
#pragma unroll
        for (int sp = 0; sp < NPB; ++sp)
#pragma unroll
            for (int dt = 0; dt < ND; ++dt) {
                const char* b = vsl + 16 * sp * HD * 2;
                const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + voff[0][dt]));
                const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + voff[1][dt]));
                const s16x8 av = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
                if constexpr (MR == 32) acc_o[dt] = DT<T>::mfma32(__builtin_bit_cast(V8, av), pb[sp], acc_o[dt]);
                else acc_o[dt] = dec_mfma16<T>(__builtin_bit_cast(V8, av), pb[sp], acc_o[dt]);
            }
    };

    // whole groups of RING tiles in a loop without a mid-body exit (keeps the waitcnt merge
    // exact), then the remainder, which starts again at slot 0
    int t = t_lo;
    for (; t + RING - 1 < t_hi; t += RING)
        static_for<RING>([&](auto S) { tile(S, t + decltype(S)::value); });
    static_for<RING - 1>([&](auto S) {
        if (t + decltype(S)::value < t_hi) tile(S, t + decltype(S)::value);
    });

    // ---- split partial: O (fp32, normalised, v_scale applied) + LSE; empty -> O = 0, -inf
    const float l_full = MR == 32 ? wave_sum_halves(l_run) : quad_sum16(l_run);
    const bool empty = (l_full == 0.f) || (l_full != l_full);
    const float inv = empty ? 0.f : (KV8 ? p.v_scale : 1.f) / l_full;
    if (row_ok) {
        const int64_t rid = (((int64_t)split * p.b + bidx) * p.h + head) * sq + pos;
        float* oa = p.oaccum + rid * HD;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
            for (int g = 0; g < NA / 4; ++g) {
                // O^T element (dt, 4g + v): d = 32 dt + 8 g + 4 hh + v (MR 32), 16 dt + 4 hh + v (MR 16)
                const int d = MR == 32 ? 32 * dt + 8 * g + 4 * hh : 16 * dt + 4 * hh;
                const f32x4 v = f32x4{acc_o[dt][4 * g] * inv, acc_o[dt][4 * g + 1] * inv,
                                      acc_o[dt][4 * g + 2] * inv, acc_o[dt][4 * g + 3] * inv};
                if (p.dec_ctr) {
                    // folded combine: device-coherent stores (sc1, through to memory; the
                    // merging wave may sit on another XCD, whose L2 is not this one's)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        __hip_atomic_store(oa + d + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    *reinterpret_cast<f32x4*>(oa + d) = v;
                }
            }
        const float lsev = empty ? -INFINITY : (m_run * c + __log2f(l_full)) * kLn2;
        if (hh == 0) {
            if (p.dec_ctr) __hip_atomic_store(p.lseaccum + rid, lsev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else p.lseaccum[rid] = lsev;
        }
    }
    if (!p.dec_ctr) return;

    // ---- folded combine: the last of the (b, kv head)'s splits to arrive merges its rows
    // (the reference's combine_attn_seqk_parallel, flash_fwd_kernel_hip.h:1322-1568).  The
    // partials went out as device-coherent stores; once they are complete (vmcnt counts
    // stores) the arrival is counted; the merging wave reads them with device-coherent loads.
    // No L2 write-back / invalidate fences (one per wave cost ~100 us on C5).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* ctr = p.dec_ctr + bidx * p.hk + hk_i;
    int old = 0;
    if (lane == 0) old = atomicAdd(ctr, 1);
    old = __builtin_amdgcn_readfirstlane(__shfl(old, 0));
    if (old != p.num_splits - 1) return;
    const int ns = p.num_splits;                 // <= 128 (host)
    const int64_t nrows = (int64_t)p.b * p.h * sq;
    auto rid_of = [&](int r) {
        const int rpos = r / G;
        return ((int64_t)bidx * p.h + hk_i * G + (r - rpos * G)) * sq + rpos;
    };
    // phase 1, per row: merged LSE over the splits (lanes over splits, every row's loads in
    // flight together) and each split's weight exp(lse_s - lse) -> this wave's LDS slice
    float* wbuf = reinterpret_cast<float*>(vsl);  // [row][split], 32 x 128 floats <= 2 SLICE
    constexpr int RC = MR == 32 ? 4 : 8;         // rows per chunk (bounds the registers)
    for (int r0 = 0; r0 < rows; r0 += RC) {
        float ls0[RC], ls1[RC];
#pragma unroll
        for (int u = 0; u < RC; ++u) {
            ls0[u] = ls1[u] = -INFINITY;
            if (r0 + u < rows) {
                const int64_t rid = rid_of(r0 + u);
                if (lane < ns) ls0[u] = __hip_atomic_load(p.lseaccum + lane * nrows + rid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane + 64 < ns) ls1[u] = __hip_atomic_load(p.lseaccum + (lane + 64) * nrows + rid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int u = 0; u < RC; ++u) {
            const int r = r0 + u;
            if (r >= rows) break;
            float mx = wave_max_halves(fmaxf(ls0[u], ls1[u]));
#pragma unroll
            for (int off = 16; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
            float sum = mx == -INFINITY ? 0.f : __expf(ls0[u] - mx) + __expf(ls1[u] - mx);
            sum = wave_sum_halves(sum);
#pragma unroll
            for (int off = 16; off >= 1; off >>= 1) sum += __shfl_xor(sum, off);
            const bool rempty = (mx == -INFINITY) || sum == 0.f;
            const float lse = rempty ? INFINITY : __logf(sum) + mx;
            if (lane < ns) wbuf[r * ns + lane] = rempty ? 0.f : __expf(ls0[u] - lse);
            if (lane + 64 < ns) wbuf[r * ns + lane + 64] = rempty ? 0.f : __expf(ls1[u] - lse);
            if (p.lse && lane == 0) {
                const int rpos = r / G;
                p.lse[(int64_t)bidx * p.lse_batch + (int64_t)(hk_i * G + r - rpos * G) * p.lse_head + rpos] = lse;
            }
        }
    }
    // phase 2: O = sum_s w_s O_s; lane -> 4 d values (lane & 31) of rows r0 + 2 rr + (lane >> 5)
    const int d4 = (lane & 31) * 4;
    const int hr = lane >> 5;
    for (int r0 = 0; r0 < rows; r0 += RC) {
        f32x4 acc[RC / 2];
#pragma unroll
        for (int rr = 0; rr < RC / 2; ++rr) acc[rr] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int sp = 0; sp < ns; ++sp) {
            const float* os = p.oaccum + (int64_t)sp * nrows * HD;
#pragma unroll
            for (int rr = 0; rr < RC / 2; ++rr) {
                const int r = r0 + 2 * rr + hr;
                if (r < rows && d4 < HD) {
                    const float* src = os + rid_of(r) * HD + d4;
                    f32x4 x;
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    acc[rr] += wbuf[r * ns + sp] * x;
                }
            }
        }
#pragma unroll
        for (int rr = 0; rr < RC / 2; ++rr) {
            const int r = r0 + 2 * rr + hr;
            if (r >= rows) continue;
            const int rpos = r / G;
            T* orow = reinterpret_cast<T*>(p.o) + (int64_t)bidx * p.o_batch + (int64_t)rpos * p.o_row +
                      (int64_t)(hk_i * G + r - rpos * G) * p.o_head;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (d4 + i < p.d) orow[d4 + i] = (T)acc[rr][i];
        }
    }
    if (lane == 0) atomicExch(ctr, 0);
}

}  // namespace xfa

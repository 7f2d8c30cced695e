// fmha_bwd_kernel.h — flash-attention backward for gfx950 (CDNA4).
//
// The reference ships the backward only as unbuilt code: bwd preprocess `compute_dot_do_o`
// (flash_bwd_preprocess_kernel_hip.h:59-141), main `compute_dq_dk_dv_1colblock`
// (flash_bwd_kernel_hip.h:89-724, seqk-parallel driver :755-767, fp32 dQ atomics :637),
// `convert_dQ` (flash_bwd_preprocess_kernel_hip.h:184-270) and host-side GQA reduction
// (export.cpp:1165-1168).  Same math here, re-designed for CDNA4:
//
//  * one workgroup = 256 keys (D <= 128; 128 keys for D > 128) of one (batch, kv-head); each
//    wave owns 32 (D = 64: 64) keys and keeps dK^T and dV^T of them in accumulation registers
//    while the workgroup sweeps every query head of the GQA group x 32-row query tiles —
//    dK/dV need no cross-workgroup (or host) reduction;
//  * key-on-the-lane orientation: S = Q K^T and dP = dO V^T land with the key on the MFMA
//    lane, so (after a pairwise cvt) P and dS are directly the B operands of
//    dV^T += dO^T P and dK^T += Q^T dS (v_mfma_f32_32x32x16); dO^T / Q^T come from the same
//    swizzled LDS tile through ds_read_b64_tr_b16;
//  * dS crosses LDS once (as dS^T, bf16) for dQ = dS K, computed with v_mfma_f32_16x16x32 by
//    all waves and added to an fp32 dQ accumulator with global float atomics (256 keys per
//    workgroup => 640 MFMA flops per atomic byte, cdna_hip_programming.md Appendix B), or, in
//    deterministic mode, into one of S = ceil(CUs / (b * hk)) accumulator slices (the bound of
//    export.cpp:1090-1091): workgroup (bh, s) is the slice's only writer and walks key blocks
//    s, s + S, s + 2S, ... in order (snake order over rounds), so it adds its dQ tiles by plain
//    read-modify-write (16-byte loads and stores, D <= 128; its first block writes instead of
//    adding, so the slices need no zeroing), retires each block's stores before the next, and
//    the convert kernel sums the slices in order - bitwise reproducible, workspace independent
//    of seqlen_k;
//  * P is recomputed from the forward LSE; D = rowsum(dO*O) comes from the preprocess kernel.
#pragma once

#include "fmha_common.h"
#ifndef XFA_BWD_ABL
#define XFA_BWD_ABL 0   // (timing ablation builds only, tools/quick_variant.py: results INVALID)
#endif
#ifndef XFA_RMW_EARLY
#define XFA_RMW_EARLY 1
#endif
#ifndef XFA_BWD_RMW
#define XFA_BWD_RMW 1   // (A/B builds only: 0 = deterministic slices by float atomics)
#endif

namespace xfa {

// Waves per workgroup.  D = 128: 8 waves x 32 keys, two waves per SIMD (256 registers each)
// so one wave's LDS / global waits hide behind the other's MFMAs.  D = 64: 4 waves x 64 keys,
// one wave per SIMD with 512 registers (a 32-row D=64 Q tile has too few 16-byte chunks for
// 512 threads).
template <int HD> constexpr int bwd_waves() { return HD == 128 ? 8 : 4; }
// Keys per workgroup: 256, or 128 for D = 129..256 (4 waves x 32 keys: the 32 x 256 dK^T and
// dV^T accumulators take 256 of a wave's 512 registers).
template <int HD> constexpr int bwd_block_n() { return HD > 128 ? 128 : 256; }
// D > 128: each wave's V rows (only ever read by that wave, for dP = dO V^T) stay in registers
// for the whole sweep instead of LDS, so K, Q, dO and dS^T fit the 160 KiB
template <int HD> constexpr bool bwd_v_in_regs() { return HD > 128; }
template <int HD> constexpr size_t bwd_smem_bytes() {
    return (bwd_v_in_regs<HD>() ? 1 : 2) * (size_t)bwd_block_n<HD>() * HD * 2 + 2 * (size_t)32 * HD * 2 +
           (size_t)bwd_block_n<HD>() * 64;
}
// Deterministic mode adds dQ by read-modify-write of its slice (D <= 128). D > 128 keeps float
// atomics into the slice, as the only deterministic instance (MASK = FEAT = true): its RMW build
// faulted on the GPU (r6, 300 x 1100 non-causal) and was not pursued — D = 256 is off the C3 path.
template <int HD> constexpr bool bwd_rmw() { return XFA_BWD_RMW && HD <= 128; }
// dQ partial sums -> the fp32 accumulator (deterministic mode: this workgroup's slice, which no
// other workgroup touches) by float atomics
__device__ __forceinline__ void dq_add(float v, __amdgpu_buffer_rsrc_t r, int off) {
#if defined(XFA_BWD_ABL) && XFA_BWD_ABL == 1
    // timing ablation only (tools/quick_variant.py, results INVALID): no dQ atomics, the value
    // kept live so the dQ phase is not optimised away
    asm volatile("" :: "v"(v), "v"(off));
    (void)r;
#else
    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, r, off, 0, 0);
#endif
}
constexpr int kBwdBlockM = 32;               // query rows per tile

typedef __attribute__((ext_vector_type(4))) float f32x4_t;

template <typename T> struct DT16;
template <> struct DT16<__bf16> {
    static __device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct DT16<_Float16> {
    static __device__ __forceinline__ f32x4 mfma16(const f16x8& a, const f16x8& b, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
};

enum { kLsdPermute = 0, kLsdVec = 1, kLsdScalar = 2 };

// dS^T tile [256 keys][32 q] bf16, 64-byte rows, 8-byte pieces of 4 q.  The tr reads of dQ
// (two 4-row blocks 8 rows apart per 32-lane half) need rows r and r + 8 on different 16-byte
// chunk pairs: the chunk takes row bit 3 in its bit 1.  The dS^T stores (ds_write_b64, 16
// lanes = 16 consecutive rows at one column, 32 banks) need the 16 pieces on 16 different
// 8-byte slots of the 128-byte bank window: row bit 0 is the address' bit 6, and rows bits 1-3
// pick the chunk's bit 0 (bit 1), its bit 1 (bit 3) and the piece within the chunk (bit 2).
// (Round 3's image flipped the chunk by bit 3 only: 4-way conflicts on every store, 11.9 % of
// the backward's LDS cycles; tools/bwd_banks.py.)
__device__ __forceinline__ int ds_off(int row, int col) {
    const int s1 = (((row >> 3) & 1) << 1) | ((row >> 1) & 1);
    const int s0 = (row >> 2) & 1;
    return row * 64 + (((col >> 3) ^ s1) << 4) + ((((col >> 2) & 1) ^ s0) << 3);
}

// ---------------------------------------------------------------- preprocess ---------------
// D[row] = sum_d dO*O (fp32), and zero the fp32 dQ accumulator row (of every slice).
template <int HD, typename T>
__global__ void __launch_bounds__(256) fmha_bwd_pre_kernel(const BwdParams p, int total_rows) {
    constexpr int TPR = HD / 8;                 // threads per (token, head) row
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int r = t / TPR;
    const int c = t % TPR;
    if (r >= total_rows) return;
    const int head = r % p.h;
    const int tok = r / p.h;                    // dense: b*sq + pos ; varlen: global token
    int bidx, pos;
    if (p.cu_seqlens_q) { bidx = 0; pos = tok; }
    else { bidx = tok / p.seqlen_q; pos = tok - bidx * p.seqlen_q; }
    const int d0 = c * 8;
    float acc = 0.f;
    if (d0 < p.d) {
        const T* o = reinterpret_cast<const T*>(p.o) + (int64_t)bidx * p.o_batch + (int64_t)pos * p.o_row +
                     (int64_t)head * p.o_head + d0;
        const T* g = reinterpret_cast<const T*>(p.dout) + (int64_t)bidx * p.do_batch +
                     (int64_t)pos * p.do_row + (int64_t)head * p.do_head + d0;
        typedef __attribute__((ext_vector_type(8))) T T8;
        const T8 ov = *reinterpret_cast<const T8*>(o);
        const T8 gv = *reinterpret_cast<const T8*>(g);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = fmaf((float)ov[j], (float)gv[j], acc);
    }
#pragma unroll
    for (int m = TPR / 2; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
    const int64_t li = (int64_t)bidx * p.lse_batch + (int64_t)head * p.lse_head + pos;
    if (c == 0) p.dsum[li] = acc;
    float* qa = p.dq_accum + (int64_t)bidx * p.acc_batch + (int64_t)head * p.acc_head +
                (int64_t)pos * p.acc_row + d0;
    // (deterministic RMW slices are initialised by their own walk: no zeroing here)
    const int ns = p.dq_slices ? (bwd_rmw<HD>() ? 0 : p.dq_slices) : 1;
    for (int s = 0; s < ns; ++s, qa += p.acc_slice) {
        *reinterpret_cast<f32x4_t*>(qa) = f32x4_t{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4_t*>(qa + 4) = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
}

// dQ = dQaccum * scale -> dtype.  Deterministic mode: dQaccum = the slices summed in slice
// order (slice s holds key blocks s, s + S, ... added in that order by one workgroup).
template <int HD, typename T>
__global__ void __launch_bounds__(256) fmha_bwd_convert_kernel(const BwdParams p, int total_rows) {
    constexpr int TPR = HD / 8;
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int r = t / TPR;
    const int c = t % TPR;
    if (r >= total_rows) return;
    const int head = r % p.h;
    const int tok = r / p.h;
    int bidx, pos;
    if (p.cu_seqlens_q) { bidx = 0; pos = tok; }
    else { bidx = tok / p.seqlen_q; pos = tok - bidx * p.seqlen_q; }
    const int d0 = c * 8;
    if (d0 >= p.d) return;
    const float* qa = p.dq_accum + (int64_t)bidx * p.acc_batch + (int64_t)head * p.acc_head +
                      (int64_t)pos * p.acc_row + d0;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = qa[j];
    for (int s = 1; s < p.dq_slices; ++s) {
        qa += p.acc_slice;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += qa[j];
    }
    typedef __attribute__((ext_vector_type(8))) T T8;
    T8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (T)(acc[j] * p.scale);
    T* dq = reinterpret_cast<T*>(p.dq) + (int64_t)bidx * p.dq_batch + (int64_t)pos * p.dq_row +
            (int64_t)head * p.dq_head + d0;
    *reinterpret_cast<T8*>(dq) = v;
}

// ---------------------------------------------------------------- main ---------------------
// One key block kb (BN keys) of one (batch, kv head) bh: dK / dV of its keys, dQ partial sums
// added into dq_base (the accumulator, or this workgroup's deterministic slice).
// RMW (deterministic mode): dq_base is a slice this workgroup alone writes, so the dQ partial
// sums are added by plain read-modify-write instead of float atomics: the tile's slice values
// are loaded at the top of the iteration (with the next tile's Q / dO) and the sums stored
// back as 16-byte rows at its end (dQ^T = K^T dS^T on the MFMA puts 4 consecutive head-dim
// columns of one query row on a lane)
template <int HD, typename T, bool MASK, bool FEAT, bool RMW = false>
__device__ __forceinline__ void bwd_key_block(const BwdParams& p, char* smem, const int bh, const int kb,
                                              float* const dq_base, const bool first = false) {
    using V8 = typename DT<T>::v8;
    constexpr int NW = bwd_waves<HD>();
    constexpr int BN = bwd_block_n<HD>();
    constexpr bool VR = bwd_v_in_regs<HD>();
    constexpr int kBwdKeysPerWave = BN / NW;   // keys owned by one wave
    // how each lane gets the LSE / D of its 4-row groups: broadcast reads of a per-wave LDS
    // slot (fewer LDS instructions than 32 ds_bpermute: +5-7% at D = 128), except in the
    // instances where the allocator then spills (measured per instance, -Rpass-analysis)
    constexpr int LSD = HD <= 64 ? kLsdVec
                      : HD <= 128 ? ((!MASK && FEAT) ? kLsdPermute : kLsdVec)
                      : (MASK ? kLsdPermute : kLsdScalar);
    constexpr int NT = NW * 64;
    constexpr int KS = kBwdKeysPerWave / 32;     // 32-key subtiles per wave
    constexpr int BQ = kBwdBlockM;
    constexpr int CPR = HD / 8;
    constexpr int NS = HD / 16;
    constexpr int ND = HD / 32;
    constexpr int KT_BYTES = BN * HD * 2;
    constexpr int QT_BYTES = BQ * HD * 2;
    constexpr int NDQ = (HD / 16) / (NW / 2);   // 16x16 dQ tiles per wave (2 query halves)
    uint64_t dseed = 0, doff = 0;                // dropout key (fmha_common.h drop_key)
    if (FEAT && p.drop) drop_key(p, dseed, doff);
    constexpr int QLD = BQ * CPR / NT;          // Q (and dO) chunks per thread
    static_assert(QLD >= 1 && BQ * CPR == QLD * NT, "Q/dO tile geometry");

    char* k_lds = smem;
    char* v_lds = smem + KT_BYTES;                   // (unused when VR)
    char* q_lds = smem + (VR ? 1 : 2) * KT_BYTES;
    char* do_lds = q_lds + QT_BYTES;
    char* ds_lds = do_lds + QT_BYTES;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
    const int lr = lane & 31;
    const int hh = lane >> 5;

    const int bidx = bh / p.hk;
    const int hk_i = bh - bidx * p.hk;
    const int n0 = kb * BN;

    int q_off = 0, sq = p.seqlen_q, k_off = 0, sk = p.seqlen_k;
    if (FEAT) {
        if (p.cu_seqlens_q) { q_off = p.cu_seqlens_q[bidx]; sq = p.cu_seqlens_q[bidx + 1] - q_off; }
        if (p.cu_seqlens_k) { k_off = p.cu_seqlens_k[bidx]; sk = p.cu_seqlens_k[bidx + 1] - k_off; }
    }
    const int diag = sk - sq;

    // query positions that can see any key of [n0, n0 + BN)
    int p_lo = 0, p_hi = sq;
    if (MASK && p.wr >= 0) p_lo = max(0, n0 - diag - p.wr);
    if (MASK && p.wl >= 0) p_hi = min(sq, n0 + BN - 1 - diag + p.wl + 1);
    const int t_lo = p_lo / BQ;
    const int ntiles = n0 < sk && p_hi > p_lo ? (p_hi + BQ - 1) / BQ - t_lo : 0;
    if constexpr (RMW) {
        // the first block of a slice's walk initialises the slice: its tiles [t_lo, t_lo +
        // ntiles) get plain stores of their sums (no read) below, every other row of the G heads
        // zeros here, so later blocks can read-modify-write any row (no zeroing pass)
        if (first) {
            constexpr int C4 = HD / 4;   // 16-byte chunks per accumulator row
            const int r0 = t_lo * BQ, r1 = min(sq, (t_lo + ntiles) * BQ);
            const int nz = ntiles ? sq - (r1 - r0) : sq;
            for (int i = threadIdx.x; i < p.group * nz * C4; i += NW * 64) {
                const int g = i / (nz * C4), rem = i - g * nz * C4;
                int row = rem / C4;
                const int c = rem - row * C4;
                if (ntiles && row >= r0) row += r1 - r0;
                float* dst = dq_base + (int64_t)bidx * p.acc_batch + (int64_t)(hk_i * p.group + g) * p.acc_head +
                             (int64_t)(q_off + row) * p.acc_row + 4 * c;
                *reinterpret_cast<f32x4_t*>(dst) = f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
        }
    }
    if (n0 >= sk) return;
    const int G = p.group;
    const int n_iter = ntiles * G;

    // ---- K and V tiles (all BN keys) -> LDS, once
    {
        const T* kb = reinterpret_cast<const T*>(p.k) + (int64_t)bidx * p.k_batch +
                      (int64_t)k_off * p.k_row + (int64_t)hk_i * p.k_head;
        const T* vb = reinterpret_cast<const T*>(p.v) + (int64_t)bidx * p.v_batch +
                      (int64_t)k_off * p.v_row + (int64_t)hk_i * p.v_head;
        for (int i = tid; i < BN * CPR; i += NT) {
            const int r = i / CPR, c = i % CPR;
            const int n = n0 + r;
            uint4 x = make_uint4(0, 0, 0, 0), y = make_uint4(0, 0, 0, 0);
            if (n < sk && c * 8 < p.d) {
                x = *reinterpret_cast<const uint4*>(kb + (int64_t)n * p.k_row + c * 8);
                y = *reinterpret_cast<const uint4*>(vb + (int64_t)n * p.v_row + c * 8);
            }
            *reinterpret_cast<uint4*>(k_lds + lds_off<HD>(r, c)) = x;
            if (!VR) *reinterpret_cast<uint4*>(v_lds + lds_off<HD>(r, c)) = y;
        }
    }
    int my_key[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) my_key[ks] = n0 + wave * kBwdKeysPerWave + 32 * ks + lr;
    // VR: this wave's V rows as the B operands of dP = dO V^T (key = lane, d chunk 2s + hh)
    V8 vfrag[VR ? NS : 1];
    if constexpr (VR) {
        static_assert(KS == 1, "V in registers: one 32-key subtile per wave");
        const T* vb = reinterpret_cast<const T*>(p.v) + (int64_t)bidx * p.v_batch +
                      (int64_t)k_off * p.v_row + (int64_t)hk_i * p.v_head;
        const __amdgpu_buffer_rsrc_t vrs = make_rsrc(vb, (uint32_t)(((int64_t)sk * p.v_row) * 2));
        const int key = my_key[0];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int col = 16 * s + 8 * hh;
            const int off = (key < sk && col < p.d) ? key * (int)p.v_row * 2 + col * 2 : kOOB;
            vfrag[s] = __builtin_bit_cast(V8, buf_load16(vrs, off));
        }
    }

    // ---- Q / dO tile loader (QLD 16-byte chunks of each per thread)
    const int lrow = tid / CPR, lcol = tid % CPR;
    constexpr int LROW_STEP = NT / CPR;
    const bool ld_ok = lcol * 8 < p.d;
    uint4 qreg[QLD], doreg[QLD];
    // LSE (lanes 0-31, pre-multiplied by log2e) and D = rowsum(dO*O) (lanes 32-63) of the
    // tile's 32 rows: one load per lane, prefetched with Q/dO, shared through LDS
    // The raw value is kept until the end of the iteration: converting it right after the
    // load makes the wave wait vmcnt on it, and vmcnt is in order, so that wait would also
    // retire the previous tile's dQ atomics (thousands of cycles with every CU issuing).
    float lsd_raw = 0.f, lsd_raw2 = 0.f;   // (masked instances: LSE in lsd_raw, D in lsd_raw2)
    bool lsd_ok = false;
    auto lsd_value = [&]() {
        const float dv = MASK ? lsd_raw2 : lsd_raw;
        return hh ? (lsd_ok ? dv : 0.f) : (lsd_ok ? lsd_raw * kLog2e : INFINITY);
    };
    auto load_q = [&](int it) {
        const int g = it / ntiles;
        const int tt = p.desc ? (g + 1) * ntiles - 1 - it : it - g * ntiles;
        const int head = hk_i * G + g;
        {
            const int pos = (t_lo + tt) * BQ + lr;
            const bool ok = pos < sq;
            const int64_t lrow = (int64_t)bidx * p.lse_batch + (int64_t)head * p.lse_head + q_off;
            if constexpr (MASK) {
                // both rows load through wave-uniform descriptors and stay raw until
                // lsd_value() picks one. A per-lane pointer select (hh ? dsum : lse) here is a
                // 64-bit VGPR the allocator spills in these instances; the scratch reload's
                // vmcnt(0) then retires the previous tile's dQ atomics every iteration (C3 +0.8 %)
                const int off = (ok ? pos : 0) * 4;
                lsd_raw = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(make_rsrc(p.lse + lrow, (uint32_t)(sq * 4)), off, 0, 0));
                lsd_raw2 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(make_rsrc(p.dsum + lrow, (uint32_t)(sq * 4)), off, 0, 0));
            } else {
                lsd_raw = (hh ? p.dsum : p.lse)[lrow + (ok ? pos : 0)];
            }
            lsd_ok = ok;
        }
        // buffer loads over this head's rows [q0, sq): rows past the end and padded head-dim
        // chunks read as zeros (no branches)
        const int q0n = (t_lo + tt) * BQ;
        const T* qb = reinterpret_cast<const T*>(p.q) + (int64_t)bidx * p.q_batch +
                      (int64_t)(q_off + q0n) * p.q_row + (int64_t)head * p.q_head;
        const T* gb = reinterpret_cast<const T*>(p.dout) + (int64_t)bidx * p.do_batch +
                      (int64_t)(q_off + q0n) * p.do_row + (int64_t)head * p.do_head;
        const int nrows = max(0, sq - q0n);
        const __amdgpu_buffer_rsrc_t qrs = make_rsrc(qb, (uint32_t)(nrows * p.q_row * 2));
        const __amdgpu_buffer_rsrc_t grs = make_rsrc(gb, (uint32_t)(nrows * p.do_row * 2));
#pragma unroll
        for (int i = 0; i < QLD; ++i) {
            const int r = lrow + i * LROW_STEP;
            const int qo = ld_ok ? r * (int)p.q_row * 2 + lcol * 16 : kOOB;
            const int go = ld_ok ? r * (int)p.do_row * 2 + lcol * 16 : kOOB;
            const u32x4 a = buf_load16(qrs, qo), b = buf_load16(grs, go);
            qreg[i] = make_uint4(a[0], a[1], a[2], a[3]);
            doreg[i] = make_uint4(b[0], b[1], b[2], b[3]);
        }
    };
    auto store_q = [&]() {
#pragma unroll
        for (int i = 0; i < QLD; ++i) {
            const int r = lrow + i * LROW_STEP;
            *reinterpret_cast<uint4*>(q_lds + lds_off<HD>(r, lcol)) = qreg[i];
            *reinterpret_cast<uint4*>(do_lds + lds_off<HD>(r, lcol)) = doreg[i];
        }
    };

    // per-lane LDS addresses (tile-relative constants fold into the ds_read offsets)
    // D = 256: the swizzle only touches chunk bits 0-3, so chunk c + 16 is the address of chunk
    // c plus 256 bytes: half the address registers (NA of NS), the rest immediate offsets
    constexpr int NA = HD > 128 ? NS / 2 : NS;
    constexpr int NTA = HD > 128 ? ND / 2 : ND;
    const char* kaddr_[NA];
    const char* qaddr_[NA];
#pragma unroll
    for (int s = 0; s < NA; ++s) {
        kaddr_[s] = k_lds + lds_off<HD>(wave * kBwdKeysPerWave + lr, 2 * s + hh);   // + 32*ks rows
        qaddr_[s] = q_lds + lds_off<HD>(lr, 2 * s + hh);
    }
    auto kaddr = [&](const int s) { return kaddr_[s % NA] + (s / NA) * 256; };
    auto qaddr = [&](const int s) { return qaddr_[s % NA] + (s / NA) * 256; };
    const int q4 = (lane & 15) >> 2;
    // LDS addresses as integers that include the LDS base of their tile, so every constant part
    // (ring row block, d tile, key subtile, dO vs Q) lands in the ds_read offset field (from a
    // pointer into smem the compiler added an SGPR base to the lane offset before every read)
    const int sbase = (int)(size_t)smem;
    constexpr int Q_OFF = (VR ? 1 : 2) * KT_BYTES, DS_OFF = Q_OFF + 2 * QT_BYTES;
    int troff_[2][NTA];   // transposed reads of the Q / dO tile (A operand: rows q, column d)
#pragma unroll
    for (int part = 0; part < 2; ++part)
#pragma unroll
        for (int dt = 0; dt < NTA; ++dt) {
            const int r = 4 * hh + q4 + 8 * part;
            const int col = 32 * dt + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
            troff_[part][dt] = sbase + Q_OFF + lds_off<HD>(r, col >> 3) + 8 * ((col >> 2) & 1);
        }
    auto troff = [&](const int part, const int dt) { return troff_[part][dt % NTA] + (dt / NTA) * 256; };
    // dQ phase (16x16x32): wave -> query half mt, d tiles
    const int mt = wave & 1;
    const int g16 = lane >> 4;
    const int p4 = lane & 3;
    const int qq = (lane & 15) >> 2;
    // tr-read bases for dQ = dS K; the swizzles only see row bits < 4, so the 32-key step
    // is a plain immediate offset (keeps the addresses out of the register budget)
    int dq_aoff[2], dq_boff[HD > 128 ? 1 : NDQ][2];
#pragma unroll
    for (int part = 0; part < 2; ++part) {
        const int kr0 = 8 * g16 + qq + 4 * part;
        dq_aoff[part] = sbase + DS_OFF + ds_off(kr0, 16 * mt + 4 * p4);
#pragma unroll
        for (int i = 0; i < (HD > 128 ? 1 : NDQ); ++i) {
            const int dcol = 16 * ((wave >> 1) * NDQ + i) + 4 * p4;
            dq_boff[i][part] = sbase + lds_off<HD>(kr0, dcol >> 3) + 8 * ((dcol >> 2) & 1);
        }
    }

    // (D > 128: the dQ K-read offsets are recomputed per use instead of held in registers)
    auto dqb = [&](const int i, const int part) {
        if constexpr (HD > 128) {
            const int kr0 = 8 * g16 + qq + 4 * part;
            const int dcol = 16 * ((wave >> 1) * NDQ + i) + 4 * p4;
            return sbase + lds_off<HD>(kr0, dcol >> 3) + 8 * ((dcol >> 2) & 1);
        } else {
            return dq_boff[i][part];
        }
    };

    f32x16 dk[KS][ND], dv[KS][ND];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) { dk[ks][dt] = f32x16{}; dv[ks][dt] = f32x16{}; }

    const float c = p.scale_log2;
    float lsd_cur = 0.f;
    float* const lsd_slot = reinterpret_cast<float*>(ds_lds + wave * kBwdKeysPerWave * 64);
    if (n_iter > 0) { load_q(0); }
    __syncthreads();                     // K tile visible
    if (n_iter > 0) { store_q(); lsd_cur = lsd_value(); }
    __syncthreads();

    for (int it = 0; it < n_iter; ++it) {
        const int g = it / ntiles;
        const int tt = p.desc ? (g + 1) * ntiles - 1 - it : it - g * ntiles;
        const int head = hk_i * G + g;
        const int q0 = (t_lo + tt) * BQ;
        // RMW: this tile's rows of the dQ slice (rows past the end / padded columns read as
        // zeros and their stores are dropped by the descriptor bounds) and this lane's offsets
        auto dq_rsrc = [&]() {
            const float* t = dq_base + (int64_t)bidx * p.acc_batch + (int64_t)head * p.acc_head +
                             (int64_t)(q_off + q0) * p.acc_row;
            return make_rsrc(t, (uint32_t)(max(0, sq - q0) * p.acc_row * 4));
        };
        auto dq_off = [&](const int i) {
            const int d = 16 * ((wave >> 1) * NDQ + i) + 4 * g16;
            return d < p.d ? (16 * mt + (lane & 15)) * (int)p.acc_row * 4 + d * 4 : kOOB;
        };
        f32x4 dq_old[RMW ? NDQ : 1];
        // this tile's LSE / D -> a private slot in this wave's own dS^T rows (nobody reads
        // them before this wave's dS^T store; the other waves' dQ reads ended at the last
        // barrier), read back below as broadcast float4s
        const float lsd = lsd_cur;
        if constexpr (LSD != kLsdPermute) lsd_slot[lane] = lsd;
        // (!VR: unconditional — the last iteration reloads its own tile — so the compiler's
        // waitcnt analysis sees the loads and their wait on every path; conditional, it kept
        // them pending across the back-edge and waited vmcnt at the loop head, retiring the
        // previous tile's dQ atomics there)
        if (!VR) load_q(min(it + 1, n_iter - 1));
        if constexpr (RMW && XFA_RMW_EARLY) {
            const __amdgpu_buffer_rsrc_t rs = dq_rsrc();
#pragma unroll
            for (int i = 0; i < NDQ; ++i)
                dq_old[i] = first || XFA_BWD_ABL == 1 ? f32x4{} : __builtin_bit_cast(f32x4, buf_load16(rs, dq_off(i)));
        }

        // ---- S = Q K^T and dP = dO V^T (key on the lane, query rows in registers)
        f32x16 s_acc[KS], dp_acc[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) { s_acc[ks] = f32x16{}; dp_acc[ks] = f32x16{}; }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const V8 qa = *reinterpret_cast<const V8*>(qaddr(s));
            const V8 ga = *reinterpret_cast<const V8*>(qaddr(s) + QT_BYTES);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const V8 kb = *reinterpret_cast<const V8*>(kaddr(s) + ks * 32 * HD * 2);
                V8 vb;
                if constexpr (VR) vb = vfrag[s];
                else vb = *reinterpret_cast<const V8*>(kaddr(s) + KT_BYTES + ks * 32 * HD * 2);
                s_acc[ks] = DT<T>::mfma32(qa, kb, s_acc[ks]);
                dp_acc[ks] = DT<T>::mfma32(ga, vb, dp_acc[ks]);
            }
            // D > 128: keep the scheduler from hoisting every k-step's LDS operands (register
            // pressure beside the 256 accumulator registers of dK^T / dV^T)
            if constexpr (HD > 128) __builtin_amdgcn_sched_barrier(0);
        }
        // (VR: the next tile's Q / dO loads go out only now, so their 32 staging registers are
        // not live across the S / dP product, the register peak)
        if (VR && it + 1 < n_iter) load_q(it + 1);
        // ---- P = exp2(S*c - LSE*log2e), dS = P * (dP - D)
        float alibi_w = 0.f;
        if (FEAT && p.alibi) alibi_w = p.alibi[bidx * p.alibi_bstride + head] * p.alibi_mul;
        // the window / key-range test only where this wave's 32 keys x the 32 rows cross an edge
        const int kw0 = n0 + wave * kBwdKeysPerWave, kw1 = kw0 + kBwdKeysPerWave - 1;
        bool need_mask = kw1 >= sk;
        if (MASK && p.wr >= 0) need_mask = need_mask || kw1 >= q0 + diag + p.wr + 1;
        if (MASK && p.wl >= 0) need_mask = need_mask || kw0 < q0 + BQ - 1 + diag - p.wl;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const int pos0 = q0 + 8 * gq + 4 * hh;
            // rows 8gq + 4hh + i of this tile: slot[row] holds its LSE, slot[32 + row] its D
            float lse4[4], d4[4];
            if constexpr (LSD == kLsdVec) {
                const f32x4 l = *reinterpret_cast<const f32x4*>(lsd_slot + 8 * gq + 4 * hh);
                const f32x4 dd = *reinterpret_cast<const f32x4*>(lsd_slot + 32 + 8 * gq + 4 * hh);
#pragma unroll
                for (int i = 0; i < 4; ++i) { lse4[i] = l[i]; d4[i] = dd[i]; }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = 8 * gq + 4 * hh + i;
                    if constexpr (LSD == kLsdScalar) {
                        lse4[i] = lsd_slot[row];
                        d4[i] = lsd_slot[32 + row];
                    } else {   // lane (row) holds its LSE, lane 32 + row its D
                        lse4[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * row, __float_as_int(lsd)));
                        d4[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * row + 128, __float_as_int(lsd)));
                    }
                }
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                // dropout: the 4 rows pos0 .. +3 of this lane's key are one Philox block
                // (fmha_common.h drop_block, the forward's draw); kept P scaled by 1 / p_keep
                u32x4 dw = u32x4{0, 0, 0, 0};
                if (FEAT && p.drop) dw = drop_block(dseed, doff, bidx * p.h + head, pos0, my_key[ks]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 4 * gq + i;
                    const int pos = pos0 + i;
                    const int key = my_key[ks];
                    float w = s_acc[ks][r];
                    float dcap = 1.f;
                    if (FEAT && p.softcap_on) { w = fast_tanh(w * p.softcap_pre); dcap = 1.f - w * w; }
                    if (FEAT && p.alibi) w -= alibi_w * (float)abs(pos + diag - key);
                    float pr = fast_exp2(fmaf(w, c, -lse4[i]));
                    if (!MASK && need_mask) {   // (unmasked instances: keys past the end only)
                        pr = (unsigned)key < (unsigned)max(sk, 0) ? pr : 0.f;
                    }
                    if (FEAT && p.drop) {
                        const bool keep = drop_keep(dw[i], key & 3, p.keep_thr);
                        s_acc[ks][r] = keep ? pr * p.rp_keep : 0.f;
                        dp_acc[ks][r] = pr * ((keep ? dp_acc[ks][r] * p.rp_keep : 0.f) - d4[i]) * dcap;
                    } else {
                        s_acc[ks][r] = pr;
                        dp_acc[ks][r] = pr * (dp_acc[ks][r] - d4[i]) * dcap;
                    }
                }
            }
        }
        // masked instances: the window / key-range mask as one wave-uniform block after the tile
        // (inside the unrolled score loop the compiler split the tile into a branch per score;
        // C3 +2.4 %): P and dS of invisible scores -> 0
        if (MASK && need_mask) {
#pragma unroll
            for (int gq = 0; gq < 4; ++gq)
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = 4 * gq + i;
                        const int pos = q0 + 8 * gq + 4 * hh + i;
                        // visible keys of row pos: [lo, hi) -> one unsigned compare
                        const int hi = (MASK && p.wr >= 0) ? min(sk, pos + diag + p.wr + 1) : sk;
                        const int lo = (MASK && p.wl >= 0) ? max(0, pos + diag - p.wl) : 0;
                        const bool vis = (unsigned)(my_key[ks] - lo) < (unsigned)max(hi - lo, 0);
                        s_acc[ks][r] = vis ? s_acc[ks][r] : 0.f;
                        dp_acc[ks][r] = vis ? dp_acc[ks][r] : 0.f;
                    }
        }
        // ---- dV^T += dO^T P ; dK^T += Q^T dS  (P / dS accumulators are the B operands)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
            const int rb = 16 * sp * HD * 2;
#pragma unroll
            for (int dt = 0; dt < ND; ++dt) {
                const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(troff(0, dt) + QT_BYTES + rb));
                const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(troff(1, dt) + QT_BYTES + rb));
                const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                const s16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(troff(0, dt) + rb));
                const s16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(troff(1, dt) + rb));
                const s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    V8 pb, sb;
#pragma unroll
                    for (int j = 0; j < 8; ++j) { pb[j] = (T)s_acc[ks][8 * sp + j]; sb[j] = (T)dp_acc[ks][8 * sp + j]; }
                    dv[ks][dt] = DT<T>::mfma32(__builtin_bit_cast(V8, av), pb, dv[ks][dt]);
                    dk[ks][dt] = DT<T>::mfma32(__builtin_bit_cast(V8, bv), sb, dk[ks][dt]);
                }
                if constexpr (HD > 128) __builtin_amdgcn_sched_barrier(0);
            }
        }
        // RMW: the slice's current values of this tile (issued after the S / dP register peak;
        // the dS^T store, the barrier and the dQ product cover their latency)
        if constexpr (RMW && !XFA_RMW_EARLY) {
            const __amdgpu_buffer_rsrc_t rs = dq_rsrc();
#pragma unroll
            for (int i = 0; i < NDQ; ++i)
                dq_old[i] = first ? f32x4{} : __builtin_bit_cast(f32x4, buf_load16(rs, dq_off(i)));
        }
        // ---- dS^T -> LDS (bf16/f16): row = key (this lane), 4 consecutive q per store
        {
            typedef __attribute__((ext_vector_type(4))) T T4;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int krow = wave * kBwdKeysPerWave + 32 * ks + lr;
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const T4 v = {(T)dp_acc[ks][4 * gq], (T)dp_acc[ks][4 * gq + 1],
                                  (T)dp_acc[ks][4 * gq + 2], (T)dp_acc[ks][4 * gq + 3]};
                    *reinterpret_cast<T4*>(ds_lds + ds_off(krow, 8 * gq + 4 * hh)) = v;
                }
            }
        }
        __syncthreads();
        // Q / dO of this tile are dead after the barrier above (dQ reads only dS^T and K)
        if (!VR || it + 1 < n_iter) store_q();
        lsd_cur = lsd_value();      // every vmcnt wait of the iteration comes before its atomics
        asm volatile("" : "+v"(lsd_cur));   // (pinned: not sunk below the atomics)
        // ---- dQ[q][d] += dS K over the 256 keys (16x16x32; A = dS via tr-read of dS^T)
        {
            f32x4 dq[NDQ];
#pragma unroll
            for (int i = 0; i < NDQ; ++i) dq[i] = f32x4{};
#pragma unroll
            for (int ks = 0; ks < BN / 32; ++ks) {
                const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(dq_aoff[0] + ks * 32 * 64));
                const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(dq_aoff[1] + ks * 32 * 64));
                const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                const V8 a = __builtin_bit_cast(V8, av);
#pragma unroll
                for (int i = 0; i < NDQ; ++i) {
                    const s16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s16x4*)(size_t)(dqb(i, 0) + ks * 32 * HD * 2));
                    const s16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s16x4*)(size_t)(dqb(i, 1) + ks * 32 * HD * 2));
                    const s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
                    // (RMW: dQ^T[d][q] = K^T dS^T, the operands swapped: a lane holds 4
                    // consecutive d of query row lane & 15)
                    if constexpr (RMW) dq[i] = DT16<T>::mfma16(__builtin_bit_cast(V8, bv), a, dq[i]);
                    else dq[i] = DT16<T>::mfma16(a, __builtin_bit_cast(V8, bv), dq[i]);
                }
                if constexpr (HD > 128) __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (RMW) {
                const __amdgpu_buffer_rsrc_t rs = dq_rsrc();
#pragma unroll
                for (int i = 0; i < NDQ; ++i) {
                    const f32x4 v = dq_old[i] + dq[i];
#if defined(XFA_BWD_ABL) && XFA_BWD_ABL == 1
                    asm volatile("" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));   // (timing ablation)
#else
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, dq_off(i), 0, 0);
#endif
                }
            } else {
            // buffer atomics over this (batch, head)'s rows [q0, sq): rows past the end and the
            // padded head-dim columns fall outside the descriptor and are dropped (no branches)
            const float* qa = dq_base + (int64_t)bidx * p.acc_batch + (int64_t)head * p.acc_head +
                              (int64_t)(q_off + q0) * p.acc_row;
            const __amdgpu_buffer_rsrc_t qrs =
                make_rsrc(qa, (uint32_t)(max(0, sq - q0) * p.acc_row * 4));
            const int arow = (int)p.acc_row * 4;
#pragma unroll
            for (int i = 0; i < NDQ; ++i) {
                const int d = 16 * ((wave >> 1) * NDQ + i) + (lane & 15);
                const int base = d < p.d ? (16 * mt + 4 * g16) * arow + d * 4 : kOOB;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    dq_add(dq[i][r], qrs, base + r * arow);
            }
            }
        }
        __syncthreads();
    }

    // ---- epilogue: dK = scale * (dK^T)^T, dV = (dV^T)^T
    typedef __attribute__((ext_vector_type(4))) T T4;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int key = my_key[ks];
        if (key >= sk) continue;
        T* dkr = reinterpret_cast<T*>(p.dk) + (int64_t)bidx * p.dk_batch + (int64_t)(k_off + key) * p.dk_row +
                 (int64_t)hk_i * p.dk_head;
        T* dvr = reinterpret_cast<T*>(p.dv) + (int64_t)bidx * p.dv_batch + (int64_t)(k_off + key) * p.dv_row +
                 (int64_t)hk_i * p.dv_head;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int d = 32 * dt + 8 * gq + 4 * hh;
                if (d < p.d) {
                    const T4 kv = {(T)(dk[ks][dt][4 * gq] * p.scale), (T)(dk[ks][dt][4 * gq + 1] * p.scale),
                                   (T)(dk[ks][dt][4 * gq + 2] * p.scale), (T)(dk[ks][dt][4 * gq + 3] * p.scale)};
                    const T4 vv = {(T)dv[ks][dt][4 * gq], (T)dv[ks][dt][4 * gq + 1],
                                   (T)dv[ks][dt][4 * gq + 2], (T)dv[ks][dt][4 * gq + 3]};
                    *reinterpret_cast<T4*>(dkr + d) = kv;
                    *reinterpret_cast<T4*>(dvr + d) = vv;
                }
            }
    }
}

template <int HD, typename T, bool MASK, bool FEAT, bool DET = false>
__global__ void __launch_bounds__(bwd_waves<HD>() * 64, bwd_waves<HD>() / 4) fmha_bwd_kernel(const BwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int BN = bwd_block_n<HD>();
    const int nkb = (p.seqlen_k + BN - 1) / BN;
    if constexpr (DET) {
        // workgroup (bh, s) alone owns dQ slice s and walks the key blocks of round r = 0, 1, ...
        // in order: block r*S + s in even rounds, r*S + S-1-s in odd ones (S = gridDim.y
        // slices; the snake evens out the causal work per slice). Its dQ adds are plain
        // read-modify-writes of the slice; each block's stores are retired (vmcnt(0)) before the
        // next block reads the same rows, so every dQ element receives its adds in key-block
        // order from one lane
        const int S = (int)gridDim.y, s = (int)blockIdx.y;
        float* const slice = p.dq_accum + (int64_t)s * p.acc_slice;
        for (int r = 0;; ++r) {
            const int kb = r * S + ((r & 1) ? S - 1 - s : s);
            if (kb >= nkb) break;
            if (r) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
            bwd_key_block<HD, T, MASK, FEAT, bwd_rmw<HD>()>(p, smem, (int)blockIdx.x, kb, slice, r == 0);
        }
    } else {
        // order 1: workgroup w runs on XCD w % 8 (dispatch round-robin); XCD x takes the kv
        // heads bh = x (mod 8), each with its key blocks consecutive, heaviest (causal) first
        int bh = blockIdx.x, kb = blockIdx.y;
        if (p.order) {
            const int i = (int)(blockIdx.x >> 3);
            bh = (int)(blockIdx.x & 7) + 8 * (i / nkb);
            kb = i - (i / nkb) * nkb;
        }
        bwd_key_block<HD, T, MASK, FEAT>(p, smem, bh, kb, p.dq_accum);
    }
}

}  // namespace xfa

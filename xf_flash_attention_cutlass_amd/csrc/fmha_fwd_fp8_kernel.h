// fmha_fwd_fp8_kernel.h — fp8 (OCP e4m3fn) Q/K/V forward for gfx950: both GEMMs on the
// block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4 (E8M0 scales fixed at 1.0), which runs at
// twice the bf16 rate (MI355X_MICROARCH.md § Matrix cores).
//
// The reference's MMA atoms are fp16/bf16 only (mma_gfx928_hip.hpp:146,182); this path is the
// north_star's "two back-to-back GEMMs on ... fp8 MFMA".  Semantics = the bf16 forward on the
// dequantised inputs Q = q8 * q_scale, K = k8 * k_scale, V = v8 * v_scale (per-tensor fp32
// descales, FA3-style), with P rounded to e4m3 for the PV product as the reference rounds P to
// the input dtype (flash_fwd_kernel_hip.h `convert_type`).
//
// Structure (one workgroup = NW waves x 32 query rows, persistent XCD-paired items, as
// fmha_fwd_kernel.h):
//  * S^T = K Q^T: the 32x32x64 A operand is 32 bytes of one key row per lane (d = 64 s + 32 h
//    .. +31 for lane half h), B the same bytes of one query row (held in registers per item).
//    A and B use the same (lane half, byte) -> k map (verified with one-hot operands,
//    tools/probe_fp8.hip), so any consistent d order contracts correctly;
//  * P: exp2 of the scaled scores, fp32 row sums, cvt_pk_fp8 into 8 dwords per lane; one
//    v_permlane32_swap per dword pair regroups them so lane half h holds keys 32h .. 32h+31 in
//    natural order (the S^T accumulator gives each half 4 of every 8 keys);
//  * O^T += V^T P^T: the A operand (V^T, d on the lane) comes from ds_read_b64_tr_b8, which per
//    16-lane group reads 8 rows x 16 byte columns and hands lane i column i of the 8 rows
//    (lane 2q+p supplies row q, bytes 8p..8p+7; probed in tools/probe_fp8.hip): 4 reads give a
//    lane 32 consecutive keys of one d column;
//  * K / V tiles (64 keys x 128 B) arrive by LDS-DMA into a double buffer; the images XOR the
//    16-byte chunk by the row so both the 32-byte row reads of K and the transposed reads of V
//    are bank-conflict-free (K: chunk ^ ((row >> 1) & 7); V: chunk ^ (((row >> 1) & 3) << 1)).
#pragma once

#include "fmha_common.h"

namespace xfa {

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) int i32x2;

__device__ __forceinline__ f32x16 mfma_fp8(const i32x8& a, const i32x8& b, const f32x16& c) {
    // cbsz = blgp = 0: A and B in fp8 e4m3; opsel 0 and E8M0 scale 127 (= 2^0) for both
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

__device__ __forceinline__ int k8_off(int row, int chunk) {      // K tile image (128-B rows)
    return row * 128 + 16 * (chunk ^ ((row >> 1) & 7));
}
__device__ __forceinline__ int v8_off(int row, int chunk) {      // V tile image (128-B rows)
    return row * 128 + 16 * (chunk ^ (((row >> 1) & 3) << 1));
}

constexpr int kFp8Tile = 64 * 128;        // bytes of one K (or V) tile: 64 keys x D = 128

template <typename T, int NW, bool MASK>
__device__ __forceinline__ void fwd8_item(const FwdParams& p, char* smem, const int bh,
                                          const int m_block) {
    constexpr int HD = 128;
    constexpr int BM = NW * 32;
    constexpr int ND = HD / 32;              // 32-wide d tiles of O^T
    constexpr int TILE = kFp8Tile;
    constexpr int IPW = TILE / 1024 / NW;    // DMA wave-instructions per wave per K (V) tile
    static_assert(IPW >= 1 && IPW * 1024 * NW == TILE, "DMA geometry");
    constexpr int NBUF = 4;                  // pipeline ring (the masked loop uses buffers 0, 1)
    constexpr int VREG = NBUF * TILE;        // LDS: K tiles of buffers 0..3, then V tiles

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int lr = lane & 31;
    const int hh = lane >> 5;

    const int bidx = bh / p.hk;
    const int hk_i = bh - bidx * p.hk;
    const int sq = p.seqlen_q, sk = p.seqlen_k;
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
    const int nb_lo = n_lo / kBlockN;
    const int nb_hi = n_hi > n_lo ? (n_hi + kBlockN - 1) / kBlockN : nb_lo;

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
    // scores arrive in q8.k8 units: fold both descales into the exp2 scale
    const float c = p.scale_log2 * p.q_scale * p.k_scale;

    // ---- Q fragments: lane holds Q[row][64 s + 32 hh .. +31] (fp8 bytes) for s = 0, 1
    i32x8 qf[2];
    {
        const char* qseq = reinterpret_cast<const char*>(p.q) + (int64_t)bidx * p.q_batch;
        const uint32_t qbytes = (uint32_t)((int64_t)(sq - 1) * p.q_row + (int64_t)(p.h - 1) * p.q_head + HD);
        const __amdgpu_buffer_rsrc_t qr = make_rsrc(qseq, qbytes);
        const int qo = row_ok ? (int)((int64_t)pos * p.q_row + (int64_t)head * p.q_head) + 32 * hh : kOOB;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const u32x4 a = buf_load16(qr, qo + 64 * s), b = buf_load16(qr, qo + 64 * s + 16);
            qf[s] = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
        }
    }

    // ---- K / V tiles by LDS-DMA: piece g (8 rows x 8 chunks) of a tile, lane l lands at
    // g KiB + 16 l, i.e. row 8 g + l / 8, image chunk l % 8, fetched from the source chunk the
    // image XOR places there
    const char* kseq = reinterpret_cast<const char*>(p.k) + (int64_t)bidx * p.k_batch + (int64_t)hk_i * p.k_head;
    const char* vseq = reinterpret_cast<const char*>(p.v) + (int64_t)bidx * p.v_batch + (int64_t)hk_i * p.v_head;
    const uint32_t kbytes = (uint32_t)((int64_t)(sk > 0 ? sk - 1 : 0) * p.k_row + HD);
    const uint32_t vbytes = (uint32_t)((int64_t)(sk > 0 ? sk - 1 : 0) * p.v_row + HD);
    const __amdgpu_buffer_rsrc_t krs = make_rsrc(kseq, kbytes);
    const __amdgpu_buffer_rsrc_t vrs = make_rsrc(vseq, vbytes);
    int dma_k[IPW], dma_v[IPW];
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
        const int g = wave * IPW + i;
        const int r = 8 * g + (lane >> 3);
        dma_k[i] = r * (int)p.k_row + 16 * ((lane & 7) ^ ((r >> 1) & 7));
        dma_v[i] = r * (int)p.v_row + 16 * ((lane & 7) ^ (((r >> 1) & 3) << 1));
    }
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    typedef __attribute__((address_space(3))) void lds_void;
    auto dma_tile = [&](const int nb, const int buf) {
        const int kso = nb * kBlockN * (int)p.k_row, vso = nb * kBlockN * (int)p.v_row;
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int g = wave_u * IPW + i;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (lds_void*)(smem + buf * TILE + g * 1024), 16, dma_k[i], kso, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lds_void*)(smem + VREG + buf * TILE + g * 1024), 16, dma_v[i], vso, 0, 0);
        }
    };
    // counted vmcnt (the DMA writes are invisible to the compiler's waitcnt tracking): all of
    // this wave's DMA landed, or all but the youngest tile's; then the workgroup barrier
    constexpr int NDMA = 2 * IPW;            // vmem instructions per tile per wave
    auto publish = [&](const bool one_in_flight = false) {
        if (one_in_flight) __builtin_amdgcn_s_waitcnt(waitcnt_vm(NDMA));
        else __builtin_amdgcn_s_waitcnt(0x0F70);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // ---- per-lane LDS read addresses: K rows (32 bytes at chunk 4 s + 2 hh + u), V^T columns
    int kaddr[2][2], vaddr[ND];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) kaddr[s][u] = (int)(size_t)smem + k8_off(lr, 4 * s + 2 * hh + u);
    {
        const int i = lane & 15, q = i >> 1, pb8 = i & 1, g = (lane >> 4) & 1;
        const int r = 32 * hh + q;                       // + 8 kb (an immediate: the swizzle
#pragma unroll                                            //   only sees row bits 1-2)
        for (int dt = 0; dt < ND; ++dt)
            vaddr[dt] = (int)(size_t)smem + VREG + v8_off(r, 2 * dt + g) + 8 * pb8;
    }
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    typedef __attribute__((address_space(3))) i32x2 lds_i32x2;
    auto rd_k = [&](const int buf, const int kt, const int s) {
        const u32x4 a = *(const lds_u32x4*)(size_t)(kaddr[s][0] + buf * TILE + kt * 32 * 128);
        const u32x4 b = *(const lds_u32x4*)(size_t)(kaddr[s][1] + buf * TILE + kt * 32 * 128);
        return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
    };
    auto rd_v = [&](const int buf, const int dt) {
        i32x8 r;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            const i32x2 t = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
                (lds_i32x2*)(size_t)(vaddr[dt] + buf * TILE + kb * 8 * 128));
            r[2 * kb] = t[0];
            r[2 * kb + 1] = t[1];
        }
        return r;
    };

    f32x16 acc_o[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) acc_o[dt] = f32x16{};
    float m_sc = -INFINITY;                 // running max in scaled (log2) units (deferred)
    float l_run = 0.f;

    auto tile = [&](const int buf, const int nb) {
        const int n0 = nb * kBlockN;
        // S^T = K Q^T: 2 key halves x 2 d halves of 64
        f32x16 st[2];
        st[0] = f32x16{};
        st[1] = f32x16{};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int s = 0; s < 2; ++s) st[kt] = mfma_fp8(rd_k(buf, kt, s), qf[s], st[kt]);
        // mask where a window edge / the end of the keys crosses this wave's rows
        if ((n0 + kBlockN > w_lr_min) || (n0 < w_ll_max)) {
#pragma unroll
            for (int v = 0; v < 32; ++v) {
                const int kt = v >> 4, r = v & 15;
                const int key = n0 + 4 * hh + 32 * kt + (r & 3) + 8 * (r >> 2);
                if (key >= my_lr || key < my_ll) st[kt][r] = -INFINITY;
            }
        }
        float mx = st[0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, st[0][r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[1][r]);
        mx = wave_max_halves(mx);
        // deferred rescale (as the bf16 kernel): m_sc moves only once a row's max passes it
        // by more than max_slack, so P <= 2^max_slack (< 448, the e4m3 maximum)
        const float m_new = fmaxf(m_sc, mx * c);
        if (__any(m_new > m_sc + p.max_slack)) {
            const float alpha = m_new == -INFINITY ? 1.f : fast_exp2(m_sc - m_new);
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < ND; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc_o[dt][r] *= alpha;
            m_sc = m_new;
        }
        const float mref = m_sc == -INFINITY ? 0.f : m_sc;
        // P = exp2(S c - m) -> e4m3, dword d of key half kt = keys 32 kt + 8 d + 4 hh + 0..3
        int pw[2][4];
        float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const float e0 = fast_exp2(__builtin_fmaf(st[kt][4 * d], c, -mref));
                const float e1 = fast_exp2(__builtin_fmaf(st[kt][4 * d + 1], c, -mref));
                const float e2 = fast_exp2(__builtin_fmaf(st[kt][4 * d + 2], c, -mref));
                const float e3 = fast_exp2(__builtin_fmaf(st[kt][4 * d + 3], c, -mref));
                rs0 += e0 + e1;
                rs1 += e2 + e3;
                int w = __builtin_amdgcn_cvt_pk_fp8_f32(e0, e1, 0, false);
                pw[kt][d] = __builtin_amdgcn_cvt_pk_fp8_f32(e2, e3, w, true);
            }
        l_run += rs0 + rs1;
        // regroup: lane half 0 keeps keys 0..31, half 1 keys 32..63 (natural order)
        i32x8 pb;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const auto r = __builtin_amdgcn_permlane32_swap((unsigned)pw[0][d], (unsigned)pw[1][d], false, false);
            pb[2 * d] = (int)r[0];        // half 0: own keys 8d + 0..3; half 1: keys 32 + 8d + 0..3
            pb[2 * d + 1] = (int)r[1];    // half 0: keys 8d + 4..7;     half 1: own 32 + 8d + 4..7
        }
        // O^T += V^T P^T
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) acc_o[dt] = mfma_fp8(rd_v(buf, dt), pb, acc_o[dt]);
    };

    // ---- tiles crossing a left window edge (and short ranges): one tile in flight, mask per wave
    auto simple_range = [&](const int lo, const int hi) {
        if (lo >= hi) return;
        dma_tile(lo, 0);
        publish();                       // also retires the Q loads
        int buf = 0;
        for (int nb = lo; nb < hi; ++nb) {
            if (nb + 1 < hi) dma_tile(nb + 1, buf ^ 1);
            const int n0 = nb * kBlockN;
            if (wave_ok && n0 < w_lr_max && n0 + kBlockN > w_ll_min) tile(buf, nb);
            publish();
            buf ^= 1;
        }
    };

    // ---- tiles every row of the workgroup sees from their left edge on: the two-stage
    // software pipeline of fmha_fwd_kernel.h.  Step j: QK^T of tile j+1 on the MFMA pipe beside
    // exp / fp32 row sums / e4m3 cvt / regroup of P_j on the VALU, then PV of tile j beside
    // X_{j+1} = S_{j+1} c - m and its row max.  K/V stream by LDS-DMA three tiles ahead through
    // 4 buffers; one barrier per tile behind a counted vmcnt.  Tiles [hm, hi) cross the right
    // edge (causal diagonal / ragged end) and are masked in registers on the way through.
    typedef __attribute__((ext_vector_type(4))) int i32x4;
    auto rd_v_asm = [&](auto OFF, const int dt) {     // V^T operand (dt), immediate buffer offset
        constexpr int off = decltype(OFF)::value;
        i32x2 t0, t1, t2, t3;
        asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(t0) : "v"(vaddr[dt]), "i"(off));
        asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(t1) : "v"(vaddr[dt]), "i"(off + 1024));
        asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(t2) : "v"(vaddr[dt]), "i"(off + 2048));
        asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(t3) : "v"(vaddr[dt]), "i"(off + 3072));
        return i32x8{t0[0], t0[1], t1[0], t1[1], t2[0], t2[1], t3[0], t3[1]};
    };
    auto lgkm_wait = [&](auto N) {
        constexpr int n = decltype(N)::value;
        __builtin_amdgcn_s_waitcnt(0xC07F | (n << 8));
        __builtin_amdgcn_sched_barrier(0);
    };
    const int lim_e = my_lr - 4 * hh;
    // Pipeline softmax without a row max per tile (the 4-wave bf16 kernel's scheme,
    // fmha_fwd4_kernel.h): P = exp2(X) against the running max m_sc; a tile whose per-lane
    // partial row sum passes 2^slack (slack <= 8: every P <= 256 < 448, the e4m3 maximum)
    // re-runs its softmax against its true row max after rescaling O and l (rare).  The
    // shifts X = S c - m and the row sums run on packed fp32 (v_pk_fma_f32 / v_pk_add_f32).
    typedef __attribute__((ext_vector_type(2))) float f2;
    const float thr = __builtin_amdgcn_exp2f(fminf(p.max_slack, 8.f));
    auto exp_dword = [&](const f32x16 (&x)[2], const int kt, const int d, f2& ra, f2& rb) {
        const float e0 = fast_exp2(x[kt][4 * d]), e1 = fast_exp2(x[kt][4 * d + 1]);
        const float e2 = fast_exp2(x[kt][4 * d + 2]), e3 = fast_exp2(x[kt][4 * d + 3]);
        ra += f2{e0, e1};
        rb += f2{e2, e3};
        const int w = __builtin_amdgcn_cvt_pk_fp8_f32(e0, e1, 0, false);
        return __builtin_amdgcn_cvt_pk_fp8_f32(e2, e3, w, true);
    };
    // the rare path: X -= its true row max (or the running max catches up), O and l rescaled,
    // P and the row sums of this tile recomputed
    auto redo = [&](f32x16 (&x)[2], int (&pw)[2][4], f2& ra, f2& rb) {
        float mx = -INFINITY;
#pragma unroll
        for (int v = 0; v < 32; ++v) mx = fmaxf(mx, x[v >> 4][v & 15]);
        mx = wave_max_halves(mx);
        const bool fresh = m_sc == -INFINITY;
        const float delta = fresh ? (mx == -INFINITY ? 0.f : mx) : fmaxf(mx, 0.f);
        const float alpha = fresh ? 1.f : fast_exp2(-delta);
        l_run *= alpha;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc_o[dt][r] *= alpha;
#pragma unroll
        for (int v = 0; v < 32; ++v) x[v >> 4][v & 15] -= delta;
        m_sc = fresh ? (mx == -INFINITY ? -INFINITY : mx) : m_sc + delta;
        ra = f2{0.f, 0.f};
        rb = f2{0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int d = 0; d < 4; ++d) pw[kt][d] = exp_dword(x, kt, d, ra, rb);
    };
    auto pipe_range = [&](const int lo, const int hm, const int hi) {
        const bool third = lo + 2 < hi;
        dma_tile(lo, 0);
        dma_tile(lo + 1, 1);
        if (third) dma_tile(lo + 2, 2);
        publish(third);
        f32x16 sa[2], sb[2];
        {   // first tile: S, mask, max, X
            sa[0] = f32x16{};
            sa[1] = f32x16{};
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int s = 0; s < 2; ++s) sa[kt] = mfma_fp8(rd_k(0, kt, s), qf[s], sa[kt]);
            if (lo >= hm) {
#pragma unroll
                for (int v = 0; v < 32; ++v) {
                    const int off = 32 * (v >> 4) + ((v & 15) & 3) + 8 * ((v & 15) >> 2);
                    if (off >= lim_e - lo * kBlockN) sa[v >> 4][v & 15] = -INFINITY;
                }
            }
            float mx = sa[0][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sa[0][r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sa[1][r]);
            mx = wave_max_halves(mx);
            const float m_new = fmaxf(m_sc, mx * c);
            if (__any(m_new > m_sc + p.max_slack)) {
                const float alpha = m_new == -INFINITY ? 1.f : fast_exp2(m_sc - m_new);
                l_run *= alpha;
#pragma unroll
                for (int dt = 0; dt < ND; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc_o[dt][r] *= alpha;
                m_sc = m_new;
            }
            const float mr = m_sc == -INFINITY ? 0.f : m_sc;
#pragma unroll
            for (int v = 0; v < 32; ++v) sa[v >> 4][v & 15] = __builtin_fmaf(sa[v >> 4][v & 15], c, -mr);
        }
        const int nsteps = hi - lo - 1;
        auto step = [&](auto KB, auto VB, auto WB, const int j, f32x16 (&st)[2], f32x16 (&sn)[2]) {
            constexpr int ks = decltype(KB)::value, vs = decltype(VB)::value, wb = decltype(WB)::value;
            const bool issue = j + 3 < hi;
            if (issue) dma_tile(j + 3, wb);
            __builtin_amdgcn_sched_barrier(0);
            // phase a: S_{j+1} (4 MFMAs) beside P_j = e4m3(exp2(X_j)), 8 values per MFMA
            sn[0] = f32x16{};
            sn[1] = f32x16{};
            int pw[2][4];
            f2 ra = {0.f, 0.f}, rb = {0.f, 0.f};
            i32x8 ka = rd_k(ks, 0, 0);
            static_for<4>([&](auto M) {
                constexpr int m = decltype(M)::value;    // MFMA m: key half m >> 1, d half m & 1
                i32x8 kn = ka;
                if constexpr (m + 1 < 4) kn = rd_k(ks, (m + 1) >> 1, (m + 1) & 1);
                sn[m >> 1] = mfma_fp8(ka, qf[m & 1], sn[m >> 1]);
                // exp values of dwords (kt = m >> 1, d = 2 (m & 1), 2 (m & 1) + 1)
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    pw[m >> 1][2 * (m & 1) + u] = exp_dword(st, m >> 1, 2 * (m & 1) + u, ra, rb);
                // keep the row-sum adds in this MFMA gap (fmha_fwd_kernel.h: else sunk below
                // phase b)
                asm volatile("" : "+v"(ra), "+v"(rb));
                ka = kn;
                __builtin_amdgcn_sched_barrier(0);
            });
            {
                const f2 rab = ra + rb;
                if (__any(rab[0] + rab[1] > thr || m_sc == -INFINITY)) {
                    asm volatile("; redo_p");
                    redo(st, pw, ra, rb);
                }
            }
            i32x8 pb;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const auto r = __builtin_amdgcn_permlane32_swap((unsigned)pw[0][d], (unsigned)pw[1][d], false, false);
                pb[2 * d] = (int)r[0];
                pb[2 * d + 1] = (int)r[1];
            }
            // phase b: O += V_j^T P_j (4 MFMAs, V^T read one MFMA ahead) beside
            // X_{j+1} = S_{j+1} c - m and its row max (8 values per MFMA)
            const float mr = m_sc == -INFINITY ? 0.f : m_sc;
            const f2 c2 = {c, c}, m2 = {-mr, -mr};
            i32x8 va = rd_v_asm(std::integral_constant<int, vs * TILE>{}, 0);
            static_for<ND>([&](auto D) {
                constexpr int dt = decltype(D)::value;
                i32x8 vn = va;
                if constexpr (dt + 1 < ND) {
                    vn = rd_v_asm(std::integral_constant<int, vs * TILE>{}, dt + 1);
                    lgkm_wait(std::integral_constant<int, 4>{});
                } else {
                    lgkm_wait(std::integral_constant<int, 0>{});
                }
                acc_o[dt] = mfma_fp8(va, pb, acc_o[dt]);
#pragma unroll
                for (int v = 8 * dt; v < 8 * dt + 8; v += 2) {
                    f2 x = {sn[v >> 4][v & 15], sn[v >> 4][(v & 15) + 1]};
                    x = __builtin_elementwise_fma(x, c2, m2);
                    sn[v >> 4][v & 15] = x[0];
                    sn[v >> 4][(v & 15) + 1] = x[1];
                }
                va = vn;
                __builtin_amdgcn_sched_barrier(0);
            });
            {
                const f2 rab = ra + rb;
                l_run += rab[0] + rab[1];
            }
            if (j + 1 >= hm) {               // edge tile: mask in registers
                const int lim_t = lim_e - (j + 1) * kBlockN;
#pragma unroll
                for (int v = 0; v < 32; ++v) {
                    const int off = 32 * (v >> 4) + ((v & 15) & 3) + 8 * ((v & 15) >> 2);
                    if (off >= lim_t) sn[v >> 4][v & 15] = -INFINITY;
                }
            }
            publish(issue);
        };
        typedef std::integral_constant<int, 0> I0;
        typedef std::integral_constant<int, 1> I1;
        typedef std::integral_constant<int, 2> I2;
        typedef std::integral_constant<int, 3> I3;
        // per-wave early exit past the causal diagonal / right window edge, as
        // fmha_fwd_kernel.h: a wave stops after the last tile any of its rows sees, drains it,
        // then keeps only its DMA share and the barriers (bit-identical results)
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
        // drain: the wave's last tile's softmax and PV (its X is in sb after an odd step count)
        // (a register copy: redo() writes it, and a runtime-selected array reference would
        // live in scratch)
        const bool odd = nsteps_w & 1;
        f32x16 sl[2] = {odd ? sb[0] : sa[0], odd ? sb[1] : sa[1]};
        int pw[2][4];
        f2 ra = {0.f, 0.f}, rb = {0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int d = 0; d < 4; ++d) pw[kt][d] = exp_dword(sl, kt, d, ra, rb);
        {
            const f2 rab = ra + rb;
            if (__any(rab[0] + rab[1] > thr || m_sc == -INFINITY)) redo(sl, pw, ra, rb);
            const f2 rab2 = ra + rb;
            l_run += rab2[0] + rab2[1];
        }
        i32x8 pb;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const auto rr = __builtin_amdgcn_permlane32_swap((unsigned)pw[0][d], (unsigned)pw[1][d], false, false);
            pb[2 * d] = (int)rr[0];
            pb[2 * d + 1] = (int)rr[1];
        }
        // V^T by the asm reads: an early-leaving wave still has DMA in flight, which the
        // builtin transposing read would make the compiler drain first
        auto pv_asm = [&](auto VB) {
            constexpr int vs = decltype(VB)::value;
            static_for<ND>([&](auto D) {
                constexpr int dt = decltype(D)::value;
                const i32x8 va = rd_v_asm(std::integral_constant<int, vs * TILE>{}, dt);
                lgkm_wait(std::integral_constant<int, 0>{});
                acc_o[dt] = mfma_fp8(va, pb, acc_o[dt]);
            });
        };
        switch (nsteps_w & 3) {
            case 0: pv_asm(I0{}); break;
            case 1: pv_asm(I1{}); break;
            case 2: pv_asm(I2{}); break;
            default: pv_asm(I3{}); break;
        }
        for (; r < nsteps; ++r) {
            const int j = lo + r;
            const bool issue = j + 3 < hi;
            if (issue) dma_tile(j + 3, (r + 3) & 3);
            publish(issue);
        }
        __syncthreads();
    };

    // tile ranges as fmha_fwd_kernel.h: [nb_lo, f_lo) cross the left window edge (simple loop);
    // [f_lo, nb_hi) run through the pipeline, [f_hi, nb_hi) masked on the way
    int f_lo = nb_hi, f_hi = nb_hi;
    {
        const int ll_max = lim_l(pos_hi), lr_min = lim_r(pos_lo);
        f_lo = max(nb_lo, (ll_max + kBlockN - 1) / kBlockN);
        f_hi = max(f_lo, min(nb_hi, lr_min / kBlockN));
        if (nb_hi - f_lo < 2) f_lo = f_hi = nb_hi;
    }
    simple_range(nb_lo, f_lo);
    if (f_lo < nb_hi) pipe_range(f_lo, f_hi, nb_hi);

    // ---- epilogue: O = v_scale * acc / l, LSE in natural units of the dequantised scores
    const float l_full = wave_sum_halves(l_run);
    const bool empty = (l_full == 0.f) || (l_full != l_full);
    const float inv = empty ? 1.f : p.v_scale / l_full;
    if (!row_ok) return;
    T* orow = reinterpret_cast<T*>(p.o) + (int64_t)bidx * p.o_batch + (int64_t)pos * p.o_row +
              (int64_t)head * p.o_head;
    store_o_row16<T, ND>(orow, acc_o, inv, HD, hh);
    if (p.lse && hh == 0)
        p.lse[(int64_t)bidx * p.lse_batch + (int64_t)head * p.lse_head + pos] =
            empty ? INFINITY : (m_sc + __log2f(l_full)) * kLn2;
}

template <typename T, int NW, bool MASK>
__global__ void __launch_bounds__(NW * 64, 2) fmha_fwd_fp8_kernel(const FwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nbh = p.b * p.hk;
    const int g = gridDim.x;
    for (int k = 0;; ++k) {
        int bh, m_block;
        if (p.persistent == 2) {         // XCD-grouped (n-1-i, i) row-block pairs (fmha_fwd_kernel.h)
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
        fwd8_item<T, NW, MASK>(p, smem, bh, m_block);
    }
}

}  // namespace xfa

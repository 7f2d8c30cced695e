// fmha_append.hip — append new K/V rows to a (paged) KV cache with optional rotary embedding,
// the KV-cache write step of `mha_fwd_kvcache`.
//
// The reference validates k/v/rotary arguments (export.cpp:1585-1669) and its kernel has the
// append + rotary code (flash_fwd_kernel_hip.h:817-934, rotary_hip.h:21-152), but its C path
// never enables it (csrc/paged_attn.cpp:513-525 forces rotary_dim 0, knew_ptr unset).  Here it
// is a separate, HBM-bound pass in front of the attention:
//
//   pos = cache_seqlens[b] + j                       (j < seqlen_new)
//   kcache[page(b, pos)][pos % page][h] = rotary(knew[b][j][h], pos)
//   vcache[...same slot...]             = vnew[b][j][h]
//   q_out[b][s][h]  = rotary(q[b][s][h], cache_seqlens[b] + (per_token ? s : 0))
//   seqlens_out[b]  = cache_seqlens[b] + seqlen_new
//
// rotary(x, pos) over the first `rdim` elements (cos/sin [seqlen_ro][rdim/2]):
//   non-interleaved (GPT-NeoX): x1 = x[i], x2 = x[i + rdim/2]  -> (x1 c - x2 s, x1 s + x2 c)
//   interleaved (GPT-J):        x1 = x[2i], x2 = x[2i + 1]      -> same, with c = cos[pos][i]
// computed in fp32 and rounded once.  One thread owns 8 output elements (16 bytes); in the
// non-interleaved case a thread of the first half also writes the partner chunk.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "fmha_launch.h"

namespace xfa {


template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&x)[8]) {
    typedef __attribute__((ext_vector_type(8))) T T8;
    const T8 v = *reinterpret_cast<const T8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (float)v[i];
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float (&x)[8]) {
    typedef __attribute__((ext_vector_type(8))) T T8;
    T8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (T)x[i];
    *reinterpret_cast<T8*>(p) = v;
}

// rotate-and-store one row (8 elements per thread; chunk c of the row)
template <typename T>
__device__ __forceinline__ void rotate_row(const AppendParams& p, const T* src, T* dst, int c,
                                           int pos) {
    const int e0 = 8 * c;
    if (e0 >= p.d) return;
    const T* cs = reinterpret_cast<const T*>(p.cos) + (int64_t)pos * (p.rdim / 2);
    const T* sn = reinterpret_cast<const T*>(p.sin) + (int64_t)pos * (p.rdim / 2);
    float x[8];
    load8(src + e0, x);
    if (e0 >= p.rdim) {                 // past the rotary part: copy
        store8(dst + e0, x);
        return;
    }
    if (p.interleaved) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float c0 = (float)cs[e0 / 2 + i], s0 = (float)sn[e0 / 2 + i];
            const float x1 = x[2 * i], x2 = x[2 * i + 1];
            x[2 * i] = x1 * c0 - x2 * s0;
            x[2 * i + 1] = x1 * s0 + x2 * c0;
        }
        store8(dst + e0, x);
        return;
    }
    const int half = p.rdim / 2;
    if (e0 >= half) return;             // written by the partner thread of the first half
    float y[8];
    load8(src + e0 + half, y);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float c0 = (float)cs[e0 + i], s0 = (float)sn[e0 + i];
        const float x1 = x[i], x2 = y[i];
        x[i] = x1 * c0 - x2 * s0;
        y[i] = x1 * s0 + x2 * c0;
    }
    store8(dst + e0, x);
    store8(dst + e0 + half, y);
}

// rows [0, n_kv) are new K/V rows (b, j, hk); rows [n_kv, n_kv + n_q) are q rows (b, s, h)
template <typename T>
__global__ void __launch_bounds__(256) fmha_append_kernel(const AppendParams p) {
    const int cpr = p.d / 8;                           // 16-byte chunks per row
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = t / cpr;
    const int c = (int)(t - row * cpr);
    const int64_t n_kv = (int64_t)p.b * p.snew * p.hk;
    const int64_t n_q = p.rdim > 0 ? (int64_t)p.b * p.sq * p.h : 0;
    if (t < p.b && p.seqlens_out) p.seqlens_out[t] = p.cache_seqlens[t] + p.snew;
    if (row < n_kv) {
        const int hki = (int)(row % p.hk);
        const int64_t bj = row / p.hk;
        const int j = (int)(bj % p.snew);
        const int bi = (int)(bj / p.snew);
        const int pos = p.cache_seqlens[bi] + j;
        // a slot past the block table's row (cache full) is dropped, never written into
        // another sequence's page
        if (pos < 0 || pos / p.page >= p.bt_stride) return;
        const int pg = p.block_table[(int64_t)bi * p.bt_stride + pos / p.page];
        const int64_t slot = (int64_t)pg * p.page_stride + (int64_t)(pos % p.page) * p.row_stride +
                             (int64_t)hki * p.head_stride;
        const int64_t src = (int64_t)bi * p.kn_batch + (int64_t)j * p.kn_row + (int64_t)hki * p.kn_head;
        const T* kn = reinterpret_cast<const T*>(p.knew) + src;
        const T* vn = reinterpret_cast<const T*>(p.vnew) + src;
        T* kc = reinterpret_cast<T*>(p.kcache) + slot;
        T* vc = reinterpret_cast<T*>(p.vcache) + slot;
        if (8 * c < p.d) {
            typedef __attribute__((ext_vector_type(8))) T T8;
            *reinterpret_cast<T8*>(vc + 8 * c) = *reinterpret_cast<const T8*>(vn + 8 * c);
            if (p.rdim > 0) rotate_row<T>(p, kn, kc, c, pos);
            else *reinterpret_cast<T8*>(kc + 8 * c) = *reinterpret_cast<const T8*>(kn + 8 * c);
        }
    } else if (row < n_kv + n_q) {
        const int64_t r = row - n_kv;
        const int hi = (int)(r % p.h);
        const int64_t bs = r / p.h;
        const int s = (int)(bs % p.sq);
        const int bi = (int)(bs / p.sq);
        const int pos = p.cache_seqlens[bi] + (p.q_per_token ? s : 0);
        const int64_t off = (int64_t)bi * p.q_batch + (int64_t)s * p.q_row + (int64_t)hi * p.q_head;
        rotate_row<T>(p, reinterpret_cast<const T*>(p.q) + off, reinterpret_cast<T*>(p.q_out) + off, c, pos);
    }
}

hipError_t launch_append(const AppendParams& p, bool fp16, hipStream_t st) {
    const int cpr = p.d / 8;
    const int64_t rows = (int64_t)p.b * p.snew * p.hk + (p.rdim > 0 ? (int64_t)p.b * p.sq * p.h : 0);
    const int64_t threads = rows * cpr > p.b ? rows * cpr : p.b;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    if (fp16) hipLaunchKernelGGL(fmha_append_kernel<_Float16>, dim3(blocks), dim3(256), 0, st, p);
    else hipLaunchKernelGGL(fmha_append_kernel<__bf16>, dim3(blocks), dim3(256), 0, st, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------- causal ALiBi LSE ------
__global__ void __launch_bounds__(256) fmha_lse_alibi_kernel(const LseAlibiParams p) {
    const int bh = blockIdx.x;
    const int bidx = bh / p.h, head = bh - bidx * p.h;
    int q_off = 0, sq = p.seqlen_q, sk = p.seqlen_k;
    if (p.cu_seqlens_q) { q_off = p.cu_seqlens_q[bidx]; sq = p.cu_seqlens_q[bidx + 1] - q_off; }
    if (p.cu_seqlens_k) sk = p.cu_seqlens_k[bidx + 1] - p.cu_seqlens_k[bidx];
    if (p.seqused_k) sk = p.seqused_k[bidx];
    if (p.leftpad_k) sk -= p.leftpad_k[bidx];
    const int pos = blockIdx.y * 256 + threadIdx.x;
    if (pos >= sq) return;
    const float slope = p.alibi[bidx * p.alibi_bstride + head];
    const int64_t i = (int64_t)bidx * p.lse_batch + (int64_t)head * p.lse_head + q_off + pos;
    const float x = p.src[i];
    p.dst[i] = isfinite(x) ? x + p.sign * slope * (float)(pos + sk - sq) : x;
}

hipError_t launch_lse_alibi(const LseAlibiParams& p, hipStream_t st) {
    const int max_sq = p.seqlen_q;     // (varlen: max_seqlen_q)
    if (max_sq <= 0 || p.b * p.h <= 0) return hipSuccess;
    hipLaunchKernelGGL(fmha_lse_alibi_kernel, dim3(p.b * p.h, (max_sq + 255) / 256), dim3(256), 0, st, p);
    return hipGetLastError();
}

}  // namespace xfa

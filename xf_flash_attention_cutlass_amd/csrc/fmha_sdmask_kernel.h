// fmha_sdmask_kernel.h — return_softmax with dropout: the materialised dropped-out softmax.
//
// The reference's forward writes S_dmask [b, h, round128(sq), round128(sk)] when
// return_softmax is set with p_dropout > 0 (flash_fwd_kernel_hip.h, apply_dropout with
// encode_dropout_in_sign_bit): P with the dropped entries' sign flipped.  Here P is the
// normalised softmax exp(s - LSE) (the reference stores it against a running max; its test
// renormalises, test.py:485-546), recomputed after the forward from Q, K and the forward's LSE,
// with the keep bit of every score drawn exactly as the forward / backward kernels draw it
// (fmha_common.h drop_block).  Positions past the sequence are 0.  A diagnostics path for small
// shapes (one thread per score, the full QK^T dot product in fp32).
#pragma once

#include "fmha_common.h"

namespace xfa {

template <typename T>
__global__ void __launch_bounds__(256) fmha_sdmask_kernel(const FwdParams p, T* s, int64_t s_batch,
                                                          int64_t s_head, int sk_r) {
    const int bh = blockIdx.x;
    const int bidx = bh / p.h, head = bh - bidx * p.h;
    const int hk_i = head / p.group;
    const int pos = blockIdx.y;
    int q_off = 0, sq = p.seqlen_q, k_off = 0, sk = p.seqlen_k;
    if (p.cu_seqlens_q) { q_off = p.cu_seqlens_q[bidx]; sq = p.cu_seqlens_q[bidx + 1] - q_off; }
    if (p.cu_seqlens_k) { k_off = p.cu_seqlens_k[bidx]; sk = p.cu_seqlens_k[bidx + 1] - k_off; }
    if (p.seqused_k) sk = p.seqused_k[bidx];
    const int diag = sk - sq;
    const int lim_r = p.wr >= 0 ? min(sk, pos + diag + p.wr + 1) : sk;
    const int lim_l = p.wl >= 0 ? max(0, pos + diag - p.wl) : 0;
    T* srow = s + (int64_t)bidx * s_batch + (int64_t)head * s_head + (int64_t)pos * sk_r;
    const T* qrow = reinterpret_cast<const T*>(p.q) + (int64_t)bidx * p.q_batch +
                    (int64_t)(q_off + pos) * p.q_row + (int64_t)head * p.q_head;
    const float lse2 = pos < sq && p.lse
        ? p.lse[(int64_t)bidx * p.lse_batch + (int64_t)head * p.lse_head + q_off + pos] * 1.4426950408889634f
        : 0.f;
    const float alibi_w = p.alibi ? p.alibi[bidx * p.alibi_bstride + head] * p.alibi_mul : 0.f;
    uint64_t dseed, doff;
    drop_key(p, dseed, doff);
    for (int key = threadIdx.x; key < sk_r; key += blockDim.x) {
        float val = 0.f;
        if (pos < sq && key < sk) {
            float pr = 0.f;
            if (key >= lim_l && key < lim_r) {
                const T* krow = reinterpret_cast<const T*>(p.k) + (int64_t)bidx * p.k_batch +
                                (int64_t)(k_off + key) * p.k_row + (int64_t)hk_i * p.k_head;
                float dot = 0.f;
                for (int d = 0; d < p.d; ++d) dot += (float)qrow[d] * (float)krow[d];
                float w = dot;
                if (p.softcap_pre > 0.f) w = tanhf(w * p.softcap_pre);
                if (p.alibi) w -= alibi_w * (float)abs(pos + diag - key);
                pr = exp2f(w * p.scale_log2 - lse2);
            }
            const u32x4 blk = drop_block(dseed, doff, bidx * p.h + head, pos, key);
            const bool keep = !p.drop || drop_keep(blk[pos & 3], key & 3, p.keep_thr);
            val = keep ? pr : -pr;
        }
        srow[key] = (T)val;
    }
}

}  // namespace xfa

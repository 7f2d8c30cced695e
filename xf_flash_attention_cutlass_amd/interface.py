"""Python wrappers over the `paged_attn` module, mirroring the reference's test.py:41-245.

Signatures and argument mapping follow the reference wrappers (softmax_scale default
D^-0.5, `maybe_contiguous`, int `cache_seqlens` broadcast to an int32 tensor), extended with
autograd: the backward runs the gfx950 bwd kernels through `paged_attn.bwd` /
`paged_attn.varlen_bwd` (the reference's `bwd` binding is commented out, export.cpp:1761).
"""
from __future__ import annotations

from typing import Optional, Union

import torch

from . import paged_attn


def _maybe_contiguous(x):
    return x.contiguous() if x is not None and x.stride(-1) != 1 else x


class _FlashAttnFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, dropout_p, softmax_scale, causal, window_size, softcap,
                alibi_slopes, deterministic, return_softmax):
        q, k, v = (_maybe_contiguous(x) for x in (q, k, v))
        out, q_p, k_p, v_p, out_p, lse, s_dmask, rng = paged_attn.fwd(
            q, k, v, None, alibi_slopes, dropout_p, softmax_scale, causal, window_size[0],
            window_size[1], softcap, return_softmax and dropout_p > 0, None)
        ctx.save_for_backward(q_p, k_p, v_p, out_p, lse, rng)
        ctx.args = (dropout_p, softmax_scale, causal, window_size, softcap, alibi_slopes,
                    deterministic, q.shape[-1])
        return out, lse, s_dmask

    @staticmethod
    def backward(ctx, dout, *_):
        q, k, v, out, lse, rng = ctx.saved_tensors
        dropout_p, scale, causal, window, softcap, alibi, deterministic, d_og = ctx.args
        dq, dk, dv, _ = paged_attn.bwd(_maybe_contiguous(dout), q, k, v, out, lse, None, None,
                                       None, alibi, dropout_p, scale, causal, window[0],
                                       window[1], softcap, deterministic, None, rng)
        dq, dk, dv = dq[..., :d_og], dk[..., :d_og], dv[..., :d_og]
        return dq, dk, dv, None, None, None, None, None, None, None, None


def flash_attn_func(q, k, v, dropout_p=0.0, causal=False, window_size=(-1, -1), softcap=0.0,
                    alibi_slopes=None, deterministic=False, return_attn_probs=False, *,
                    softmax_scale=None, q_descale=None, k_descale=None, v_descale=None,
                    out_dtype=torch.bfloat16):
    """q [b, sq, h, d], k/v [b, sk, hk, d] -> out [b, sq, h, d] (test.py:41-72).

    Extension: float8_e4m3fn q/k/v (with per-tensor descales, value = stored x descale) run the
    fp8-MFMA forward (forward only, d = 128, no ALiBi / softcap / dropout); out is `out_dtype`."""
    if softmax_scale is None:
        softmax_scale = q.shape[-1] ** (-0.5)
    if q.dtype == torch.float8_e4m3fn:
        # the fp8 forward has no dropout / softcap / ALiBi: refuse instead of dropping them
        if dropout_p != 0.0 or softcap != 0.0 or alibi_slopes is not None:
            raise NotImplementedError("fp8 q/k/v: dropout, softcap and ALiBi are not supported "
                                      f"(dropout_p={dropout_p}, softcap={softcap}, "
                                      f"alibi={'set' if alibi_slopes is not None else None})")
        out, lse = flash_attn_fp8_func(q, k, v, q_descale, k_descale, v_descale, softmax_scale,
                                       causal, window_size, out_dtype, return_lse=True)
        return out if not return_attn_probs else (out, lse, None)
    out, lse, s_dmask = _FlashAttnFunc.apply(q, k, v, dropout_p, softmax_scale, causal,
                                             tuple(int(w) for w in window_size), softcap,
                                             alibi_slopes, deterministic, return_attn_probs)
    return out if not return_attn_probs else (out, lse, s_dmask)


def flash_attn_fp8_func(q, k, v, q_descale=None, k_descale=None, v_descale=None,
                        softmax_scale=None, causal=False, window_size=(-1, -1),
                        out_dtype=torch.bfloat16, return_lse=False):
    """fp8 e4m3fn q [b, sq, h, 128], k/v [b, sk, hk, 128] with per-tensor descales (floats or
    one-element tensors; None = 1.0): both GEMMs on the gfx950 fp8 MFMA.  Forward only."""
    if q.requires_grad or k.requires_grad or v.requires_grad:
        raise NotImplementedError("the fp8 forward has no backward")
    if out_dtype not in (torch.bfloat16, torch.float16):
        raise ValueError("out_dtype must be bfloat16 or float16")
    if softmax_scale is None:
        softmax_scale = q.shape[-1] ** (-0.5)

    def _f(x):
        return 1.0 if x is None else float(x)
    q, k, v = (_maybe_contiguous(x) for x in (q, k, v))
    out, lse = paged_attn.fwd_fp8(q, k, v, None, _f(q_descale), _f(k_descale), _f(v_descale),
                                  softmax_scale, causal, int(window_size[0]), int(window_size[1]),
                                  out_dtype == torch.float16)
    return (out, lse) if return_lse else out


def flash_attn_kvpacked_func(q, kv, dropout_p=0.0, softmax_scale=None, causal=False,
                             window_size=(-1, -1), softcap=0.0, alibi_slopes=None,
                             deterministic=False, return_softmax=False):
    """kv [b, sk, 2, hk, d] (test.py:74-100)."""
    return flash_attn_func(q, kv[:, :, 0], kv[:, :, 1], dropout_p, causal, window_size, softcap,
                           alibi_slopes, deterministic, return_softmax,
                           softmax_scale=softmax_scale)


class _FlashAttnVarlenFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, max_q, max_k, dropout_p, softmax_scale, causal,
                window_size, softcap, alibi_slopes, deterministic, return_softmax, block_table):
        q, k, v = (_maybe_contiguous(x) for x in (q, k, v))
        out, q_p, k_p, v_p, out_p, lse, s_dmask, rng = paged_attn.varlen_fwd(
            q, k, v, None, cu_q, cu_k, None, block_table, alibi_slopes, max_q, max_k, dropout_p,
            softmax_scale, False, causal, window_size[0], window_size[1], softcap,
            return_softmax and dropout_p > 0, None)
        ctx.save_for_backward(q_p, k_p, v_p, out_p, lse, cu_q, cu_k, rng)
        ctx.args = (max_q, max_k, dropout_p, softmax_scale, causal, window_size, softcap,
                    alibi_slopes, deterministic, q.shape[-1], block_table is not None)
        return out, lse, s_dmask

    @staticmethod
    def backward(ctx, dout, *_):
        q, k, v, out, lse, cu_q, cu_k, rng = ctx.saved_tensors
        (max_q, max_k, dropout_p, scale, causal, window, softcap, alibi, deterministic, d_og,
         paged) = ctx.args
        if paged:
            raise RuntimeError("backward through a paged K/V cache is not supported")
        dq, dk, dv, _ = paged_attn.varlen_bwd(_maybe_contiguous(dout), q, k, v, out, lse, None,
                                              None, None, cu_q, cu_k, alibi, max_q, max_k,
                                              dropout_p, scale, False, causal, window[0],
                                              window[1], softcap, deterministic, None, rng)
        dq, dk, dv = dq[..., :d_og], dk[..., :d_og], dv[..., :d_og]
        return (dq, dk, dv) + (None,) * 13


def flash_attn_varlen_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                           dropout_p=0.0, softmax_scale=None, causal=False,
                           window_size=(-1, -1), softcap=0.0, alibi_slopes=None,
                           deterministic=False, return_attn_probs=False, block_table=None):
    """Packed q [total_q, h, d], k/v [total_k, hk, d], cu_seqlens int32 (test.py:102-149)."""
    if softmax_scale is None:
        softmax_scale = q.shape[-1] ** (-0.5)
    out, lse, s_dmask = _FlashAttnVarlenFunc.apply(
        q, k, v, cu_seqlens_q, cu_seqlens_k, int(max_seqlen_q), int(max_seqlen_k), dropout_p,
        softmax_scale, causal, tuple(int(w) for w in window_size), softcap, alibi_slopes,
        deterministic, return_attn_probs, block_table)
    return out if not return_attn_probs else (out, lse, s_dmask)


def flash_attn_varlen_kvpacked_func(q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
                                    max_seqlen_k, dropout_p=0.0, softmax_scale=None,
                                    causal=False, window_size=(-1, -1), softcap=0.0,
                                    alibi_slopes=None, deterministic=False,
                                    return_attn_probs=False):
    """kv [total_k, 2, hk, d] (test.py:151-187)."""
    return flash_attn_varlen_func(q, kv[:, 0], kv[:, 1], cu_seqlens_q, cu_seqlens_k,
                                  max_seqlen_q, max_seqlen_k, dropout_p, softmax_scale, causal,
                                  window_size, softcap, alibi_slopes, deterministic,
                                  return_attn_probs)


def flash_attn_with_kvcache(q, k_cache, v_cache, k=None, v=None, rotary_cos=None,
                            rotary_sin=None,
                            cache_seqlens: Optional[Union[int, torch.Tensor]] = None,
                            cache_batch_idx: Optional[torch.Tensor] = None,
                            cache_leftpad: Optional[torch.Tensor] = None,
                            block_table: Optional[torch.Tensor] = None, softmax_scale=None,
                            causal=False, window_size=(-1, -1), softcap=0.0,
                            rotary_interleaved=True, alibi_slopes=None, num_splits=0,
                            return_softmax_lse=False, k_scale=1.0, v_scale=1.0):
    """Decode / chunked prefill against a (paged) KV cache (test.py:189-245).  With k/v the new
    rows are first written into the cache in place at cache_seqlens (rotary_cos/sin: rotary
    embedding on k and q, interleaved = GPT-J pairs), then attended over.

    Extension: a `torch.float8_e4m3fn` paged cache is read natively (dequantised in-kernel as
    fp8 * k_scale / v_scale); it requires `block_table` and `cache_seqlens`."""
    assert k_cache.stride(-1) == 1, "k_cache must have contiguous last dimension"
    assert v_cache.stride(-1) == 1, "v_cache must have contiguous last dimension"
    if cache_leftpad is not None and (block_table is not None or k_cache.dtype == torch.float8_e4m3fn):
        raise NotImplementedError("cache_leftpad needs a non-paged cache (flash-attn: no Paged KV "
                                  "and leftpad_k at the same time)")
    q, k, v = (_maybe_contiguous(x) for x in (q, k, v))
    if softmax_scale is None:
        softmax_scale = q.shape[-1] ** (-0.5)
    if k_cache.dtype == torch.float8_e4m3fn:
        if block_table is None or cache_seqlens is None or k is not None or alibi_slopes is not None \
                or softcap > 0:
            raise NotImplementedError("fp8 K/V cache: paged decode with block_table and "
                                      "cache_seqlens only")
        if isinstance(cache_seqlens, int):
            cache_seqlens = torch.full((q.shape[0],), cache_seqlens, dtype=torch.int32,
                                       device=q.device)
        out, lse = paged_attn.fwd_kvcache_fp8(q, k_cache.view(torch.uint8),
                                              v_cache.view(torch.uint8), cache_seqlens,
                                              block_table, float(k_scale), float(v_scale),
                                              softmax_scale, causal, int(window_size[0]),
                                              int(window_size[1]), num_splits)
        return (out, lse) if return_softmax_lse else out
    if cache_seqlens is not None and isinstance(cache_seqlens, int):
        cache_seqlens = torch.full((q.shape[0],), cache_seqlens, dtype=torch.int32,
                                   device=k_cache.device)
        cache_seqlens = _maybe_contiguous(cache_seqlens)
    cache_batch_idx = _maybe_contiguous(cache_batch_idx)
    block_table = _maybe_contiguous(block_table)
    out, lse = paged_attn.fwd_kvcache(q, k_cache, v_cache, k, v, cache_seqlens, rotary_cos,
                                      rotary_sin, cache_batch_idx, block_table, alibi_slopes,
                                      None, softmax_scale, causal, int(window_size[0]),
                                      int(window_size[1]), softcap, rotary_interleaved,
                                      num_splits, _maybe_contiguous(cache_leftpad))
    return (out, lse) if return_softmax_lse else out

"""CPU oracle for the fused attention hot path — TEST INFRASTRUCTURE ONLY.

This module is a restatement (not a copy) of the reference's PyTorch oracle in
`/root/reference/test.py`, which is the only correctness authority the reference
has (its HIP kernels are DCU/gfx928-only and cannot be built or run on ROCm 7.2 /
MI355X).  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import it; the product path never does.

Functions and the reference lines they restate:

* `local_mask`          -> `construct_local_mask`          test.py:275-307
* `alibi_bias`          -> `attn_bias_from_alibi_slopes`   test.py:247-273
* `attention_ref`       -> `attention_ref`                 test.py:310-397
* `attention_lse_ref`   -> the log-sum-exp the fwd kernel writes
                           (softmax_hip.h:129-189 `normalize_softmax_lse`;
                           empty rows -> +inf, flash_fwd_kernel_hip.h:626-670)
* `random_padding_mask` -> `generate_random_padding_mask`  test.py:587-600
* `unpad_input`/`pad_input` -> flash_attn.bert_padding (third-party, not
                           vendored; semantics as used at test.py:620-635:
                           4-tuple (x_unpad, indices, cu_seqlens int32, max_seqlen))
* `block_kvcache`       -> `_generate_block_kvcache`       test.py:1597-1621
* `attention_fp8_pt`    -> no reference counterpart (the reference has no fp8 path): the
                           low-precision estimate for the fp8 Q/K/V forward, i.e. attention_ref
                           over the dequantised inputs with P rounded to e4m3 before PV, the fp8
                           analogue of the reference's rounding of P to the input dtype.  Parity
                           for the fp8 forward is therefore pinned only by this restatement.
* `apply_rotary`        -> flash_attn.layers.rotary.apply_rotary_emb (third-party, not
                           vendored; semantics as used by the commented-out rotary branch of
                           test_flash_attn_kvcache, test.py:1454-1486: GPT-NeoX halves or
                           GPT-J interleaved pairs over the first rotary_dim features,
                           positions seqlen_offsets[b] + s).  Parity for rotary is pinned only
                           by this restatement (the reference never runs it).

Pass rules (test.py:975, 1296, 1593-1594) live in `parity_ok`.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

__all__ = [
    "local_mask", "alibi_bias", "attention_ref", "attention_lse_ref",
    "random_padding_mask", "unpad_input", "pad_input", "block_kvcache",
    "parity_ok", "expand_kv", "apply_rotary", "quantize_fp8", "attention_fp8_pt",
]


def _lengths(mask: Optional[torch.Tensor], full: int):
    """Per-batch valid length broadcastable to [b, 1, 1, 1] (or the python int)."""
    if mask is None:
        return full
    return mask.sum(-1).view(-1, 1, 1, 1)


def local_mask(seqlen_q: int, seqlen_k: int, window_size=(-1, -1),
               query_padding_mask=None, key_padding_mask=None, device=None,
               key_leftpad=None) -> torch.Tensor:
    """Boolean mask, True where a (row, col) score is NOT allowed.

    Windows are bottom-right aligned: row i of a length-sq query sees keys
    [i + sk - sq - left, i + sk - sq + right] (test.py:275-307).
    """
    rows = torch.arange(seqlen_q, device=device, dtype=torch.long).view(-1, 1)
    cols = torch.arange(seqlen_k, device=device, dtype=torch.long)
    if key_leftpad is not None:
        lp = key_leftpad.view(-1, 1, 1, 1)
        cols = cols.view(1, 1, 1, -1).expand(lp.shape[0], 1, 1, seqlen_k)
        cols = torch.where(cols >= lp, cols - lp, torch.full_like(cols, 2 ** 32))
    sk = _lengths(key_padding_mask, seqlen_k)
    sq = _lengths(query_padding_mask, seqlen_q)
    left, right = int(window_size[0]), int(window_size[1])
    diag = rows + sk - sq
    if left < 0:
        return cols > diag + right
    if key_padding_mask is None:
        sk = torch.full_like(cols, seqlen_k)
    return (cols > torch.minimum(diag + right, sk)) | (cols < diag - left)


def alibi_bias(slopes: torch.Tensor, seqlen_q: int, seqlen_k: int,
               query_padding_mask=None, key_padding_mask=None, causal=False,
               key_leftpad=None) -> torch.Tensor:
    """ALiBi additive bias (test.py:247-273), broadcastable to [b, h, sq, sk]."""
    b, h = slopes.shape
    s = slopes.view(b, h, 1, 1)
    dev = slopes.device
    if causal:
        return torch.arange(-seqlen_k + 1, 1, device=dev, dtype=torch.float32) * s
    rows = torch.arange(seqlen_q, device=dev, dtype=torch.long).view(-1, 1)
    cols = torch.arange(seqlen_k, device=dev, dtype=torch.long)
    if key_leftpad is not None:
        lp = key_leftpad.view(-1, 1, 1, 1)
        cols = cols.view(1, 1, 1, -1).expand(lp.shape[0], 1, 1, seqlen_k)
        cols = torch.where(cols >= lp, cols - lp, torch.full_like(cols, 2 ** 32))
    sk = _lengths(key_padding_mask, seqlen_k)
    sq = _lengths(query_padding_mask, seqlen_q)
    dist = (rows + sk - sq - cols).abs()
    return -s * dist.to(slopes.dtype)


def alibi_bias_kernel(slopes: torch.Tensor, seqlen_q: int, seqlen_k: int, causal=False,
                      key_padding_mask=None) -> torch.Tensor:
    """ALiBi bias in the reference KERNEL's form (mask_hip.h:162-167), for the LSE the kernel
    returns: causal `+slope * col` (test.py's oracle uses slope * (col - sk + 1), a per-row
    constant apart: equal O, different LSE); otherwise `-slope * |row + sk - sq - col|`."""
    if not causal:
        return alibi_bias(slopes, seqlen_q, seqlen_k, None, key_padding_mask, causal=False)
    b, h = slopes.shape
    return torch.arange(seqlen_k, device=slopes.device, dtype=torch.float32) * slopes.view(b, h, 1, 1)


def expand_kv(x: torch.Tensor, nheads: int) -> torch.Tensor:
    """[b, s, hk, d] -> [b, s, nheads, d]; query head i reads kv head i // (nheads/hk)."""
    g = nheads // x.shape[2]
    return x.repeat_interleave(g, dim=2)


def _scores(q, k, reorder_ops: bool):
    d = q.shape[-1]
    if reorder_ops:
        return torch.einsum("bthd,bshd->bhts", q, k / math.sqrt(d))
    return torch.einsum("bthd,bshd->bhts", q / math.sqrt(d), k)


def attention_ref(q, k, v, query_padding_mask=None, key_padding_mask=None,
                  attn_bias=None, dropout_p=0.0, dropout_mask=None, causal=False,
                  window_size=(-1, -1), softcap=0.0, upcast=True,
                  reorder_ops=False, key_leftpad=None):
    """Eager attention, [b, s, h, d] layout (test.py:310-397).

    Returns (out, attention) in the input dtype.  `upcast=True` computes in fp32
    (the oracle); `upcast=False, reorder_ops=True` is the low-precision PyTorch
    estimate used by the pass rule.
    """
    if causal:
        window_size = (window_size[0], 0)
    dtype_og = q.dtype
    if upcast:
        q, k, v = q.float(), k.float(), v.float()
    sq, sk = q.shape[1], k.shape[1]
    k = expand_kv(k, q.shape[2])
    v = expand_kv(v, q.shape[2])
    scores = _scores(q, k, reorder_ops)
    if softcap > 0:
        scores = torch.tanh(scores / softcap) * softcap
    if key_padding_mask is not None:
        scores.masked_fill_(~key_padding_mask.view(key_padding_mask.shape[0], 1, 1, -1),
                            float("-inf"))
    windowed = window_size[0] >= 0 or window_size[1] >= 0
    if windowed:
        lm = local_mask(sq, sk, window_size, query_padding_mask, key_padding_mask,
                        q.device, key_leftpad=key_leftpad)
        scores.masked_fill_(lm, float("-inf"))
    if attn_bias is not None:
        scores = scores + attn_bias
    attn = torch.softmax(scores, dim=-1).to(v.dtype)
    if windowed:
        attn = attn.masked_fill(lm.all(dim=-1, keepdim=True), 0.0)
    if query_padding_mask is not None:
        attn = attn.masked_fill(~query_padding_mask.view(query_padding_mask.shape[0], 1, -1, 1), 0.0)
    drop = attn if dropout_mask is None else attn.masked_fill(~dropout_mask, 0.0)
    out = torch.einsum("bhts,bshd->bthd", drop, v * (1.0 / (1.0 - dropout_p)))
    if query_padding_mask is not None:
        out.masked_fill_(~query_padding_mask.view(query_padding_mask.shape[0], -1, 1, 1), 0.0)
    return out.to(dtype_og), attn.to(dtype_og)


def attention_lse_ref(q, k, key_padding_mask=None, attn_bias=None, causal=False,
                      window_size=(-1, -1), softcap=0.0, softmax_scale=None):
    """fp32 log-sum-exp of the masked, scaled scores: [b, h, sq].

    This is the quantity the fwd kernel writes to `softmax_lse`
    (`LSE = m*scale + log(sum)`, softmax_hip.h:129-189).  Fully masked rows give
    +inf, the kernel's empty-row convention (flash_fwd_kernel_hip.h:626-670).
    ALiBi: pass `alibi_bias_kernel(...)`, the reference kernel's form (causal
    +slope*col, mask_hip.h:163-164), which the build's LSE follows (the causal form
    of test.py:247-273 differs from it by a per-row constant that cancels in O but
    not in LSE) — see DESIGN.md §4.
    """
    if causal:
        window_size = (window_size[0], 0)
    q, k = q.float(), k.float()
    sq, sk = q.shape[1], k.shape[1]
    k = expand_kv(k, q.shape[2])
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    scores = torch.einsum("bthd,bshd->bhts", q, k) * scale
    if softcap > 0:
        scores = torch.tanh(scores / softcap) * softcap
    if key_padding_mask is not None:
        scores.masked_fill_(~key_padding_mask.view(key_padding_mask.shape[0], 1, 1, -1),
                            float("-inf"))
    if window_size[0] >= 0 or window_size[1] >= 0:
        scores.masked_fill_(local_mask(sq, sk, window_size, None, key_padding_mask, q.device),
                            float("-inf"))
    if attn_bias is not None:
        scores = scores + attn_bias
    lse = torch.logsumexp(scores, dim=-1)
    return torch.where(torch.isneginf(lse), torch.full_like(lse, float("inf")), lse)


def random_padding_mask(max_seqlen: int, batch_size: int, device=None, mode="random",
                        generator=None) -> torch.Tensor:
    """[b, max_seqlen] bool key/query padding mask (test.py:587-600)."""
    assert mode in ("full", "random", "third")
    if mode == "full":
        lengths = torch.full((batch_size, 1), max_seqlen, device=device, dtype=torch.int32)
    elif mode == "random":
        lengths = torch.randint(max(1, max_seqlen - 20), max_seqlen + 1, (batch_size, 1),
                                device=device, generator=generator)
    else:
        lengths = torch.randint(max_seqlen // 3, max_seqlen + 1, (batch_size, 1),
                                device=device, generator=generator)
    return torch.arange(max_seqlen, device=device).view(1, -1).expand(batch_size, -1) < lengths


def unpad_input(x: torch.Tensor, mask: torch.Tensor):
    """Gather the valid tokens of [b, s, ...] into [total, ...].

    Returns (x_unpad, indices, cu_seqlens int32 [b+1], max_seqlen) — the
    contract test.py:620,635 relies on (flash_attn.bert_padding.unpad_input).
    """
    lens = mask.sum(dim=-1, dtype=torch.int32)
    indices = torch.nonzero(mask.flatten(), as_tuple=False).flatten()
    cu = torch.zeros(mask.shape[0] + 1, dtype=torch.int32, device=mask.device)
    cu[1:] = torch.cumsum(lens, dim=0, dtype=torch.int32)
    flat = x.reshape(x.shape[0] * x.shape[1], *x.shape[2:])
    return flat[indices], indices, cu, int(lens.max().item())


def pad_input(x_unpad: torch.Tensor, indices: torch.Tensor, batch: int, seqlen: int):
    """Inverse of `unpad_input`: scatter [total, ...] into zeros [b, s, ...]."""
    out = torch.zeros(batch * seqlen, *x_unpad.shape[1:], dtype=x_unpad.dtype,
                      device=x_unpad.device)
    out[indices] = x_unpad
    return out.view(batch, seqlen, *x_unpad.shape[1:])


def block_kvcache(seqlen_k: int, page: int, batch: int, nheads_k: int, d: int,
                  device=None, dtype=torch.float16, generator=None):
    """Paged KV cache with a random-permutation block table (test.py:1597-1621).

    Returns (k_cache, v_cache, block_table, k_cache_paged, v_cache_paged, num_blocks):
    contiguous views [b, seqlen_k, hk, d] gathered through the table, the paged
    pools [num_blocks, page, hk, d] and block_table int32 [b, num_blocks/b].
    """
    num_blocks = math.ceil(seqlen_k / page) * batch * 3
    kp = torch.randn(num_blocks, page, nheads_k, d, device=device, dtype=dtype, generator=generator)
    vp = torch.randn(num_blocks, page, nheads_k, d, device=device, dtype=dtype, generator=generator)
    table = torch.randperm(num_blocks, dtype=torch.int32, device=device,
                           generator=generator).view(batch, -1)
    idx = table.to(torch.long).flatten()
    kc = kp[idx].reshape(batch, -1, nheads_k, d)[:, :seqlen_k]
    vc = vp[idx].reshape(batch, -1, nheads_k, d)[:, :seqlen_k]
    return kc, vc, table, kp, vp, num_blocks


def parity_ok(out, out_ref, out_pt, mult: float = 2.0, atol: float = 0.0):
    """The reference's pass rule: max|out-ref| <= mult * max|pt-ref| + atol.

    mult=2 for fwd/varlen (test.py:975, 1296), 3 (+1e-5) for kvcache
    (test.py:1593-1594), 3 for gradients (test.py:984-986).
    Returns (ok, err, bound).
    """
    err = (out.float() - out_ref.float()).abs().max().item()
    bound = mult * (out_pt.float() - out_ref.float()).abs().max().item() + atol
    return err <= bound, err, bound


def apply_rotary(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                 seqlen_offsets: torch.Tensor, interleaved: bool = False) -> torch.Tensor:
    """Rotary embedding of x [b, s, h, d] over its first 2 * cos.shape[1] features; token s of
    batch b uses row seqlen_offsets[b] + s of cos/sin ([seqlen_ro, rotary_dim / 2]).  Computed
    in fp32, returned in x's dtype (flash_attn.layers.rotary.apply_rotary_emb semantics)."""
    b, s, h, d = x.shape
    rd = 2 * cos.shape[1]
    pos = seqlen_offsets.view(-1, 1).long().cpu() + torch.arange(s).view(1, -1)   # [b, s]
    c = cos.float().cpu()[pos].unsqueeze(2)          # [b, s, 1, rd/2]
    sn = sin.float().cpu()[pos].unsqueeze(2)
    xf = x.float().cpu()
    xr = xf[..., :rd]
    if interleaved:
        x1, x2 = xr[..., 0::2], xr[..., 1::2]
        o1, o2 = x1 * c - x2 * sn, x1 * sn + x2 * c
        out = torch.stack((o1, o2), dim=-1).reshape(b, s, h, rd)
    else:
        x1, x2 = xr[..., : rd // 2], xr[..., rd // 2:]
        out = torch.cat((x1 * c - x2 * sn, x1 * sn + x2 * c), dim=-1)
    return torch.cat((out, xf[..., rd:]), dim=-1).to(x.dtype)


def quantize_fp8(x: torch.Tensor):
    """Per-tensor OCP e4m3fn quantisation: (x8, scale) with x ~ x8.float() * scale."""
    scale = float(x.float().abs().max()) / 448.0 or 1.0
    return (x.float() / scale).clamp(-448, 448).to(torch.float8_e4m3fn), scale


def attention_fp8_pt(q8, k8, v8, q_scale, k_scale, v_scale, causal=False, window_size=(-1, -1)):
    """fp32 attention over the dequantised fp8 inputs with P = exp(s - rowmax) rounded to e4m3
    before the PV product and the row sum taken over the unrounded P ([b, s, h, d] layout)."""
    q, k, v = (x.float() * s for x, s in ((q8, q_scale), (k8, k_scale), (v8, v_scale)))
    if causal:
        window_size = (window_size[0], 0)
    sq, sk = q.shape[1], k.shape[1]
    k = expand_kv(k, q.shape[2])
    v = expand_kv(v, q.shape[2])
    scores = torch.einsum("bthd,bshd->bhts", q, k) * q.shape[-1] ** -0.5
    if window_size[0] >= 0 or window_size[1] >= 0:
        scores.masked_fill_(local_mask(sq, sk, window_size, device=q.device), float("-inf"))
    m = scores.amax(-1, keepdim=True)
    m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    p = torch.exp(scores - m)
    l = p.sum(-1, keepdim=True)
    p8 = p.to(torch.float8_e4m3fn).float()
    out = torch.einsum("bhts,bshd->bthd", p8, v) / l.permute(0, 2, 1, 3).clamp_min(1e-30)
    return out

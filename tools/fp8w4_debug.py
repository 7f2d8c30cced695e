"""Diagnose the 4-wave fp8 forward (fp8_w4=1) against a plain fp32 attention on structured
inputs: where NaNs / errors sit (row within the 256-row item, lane-row within the 32-row block,
d column), so a layout or pipeline bug shows its shape.

  python tools/fp8w4_debug.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ref_attn(q, k, v, causal):
    # q [b, sq, h, d], k/v [b, sk, hk, d] fp32
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    g = h // hk
    k = k.repeat_interleave(g, dim=2)
    v = v.repeat_interleave(g, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * d ** -0.5
    if causal:
        i = torch.arange(sq)[:, None] + sk - sq
        j = torch.arange(sk)[None, :]
        s = s.masked_fill(j > i, float("-inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.softmax(s, -1)
    return torch.einsum("bhqk,bkhd->bqhd", p, v), lse


def q8(x):
    sc = float(x.abs().max()) / 448.0 or 1.0
    return (x / sc).clamp(-448, 448).to(torch.float8_e4m3fn), sc


def run(lib, name, q, k, v, causal):
    from xf_flash_attention_cutlass_amd import capi
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    (qq, qs), (kk, ks), (vv, vs) = q8(q), q8(k), q8(v)
    out = torch.full((b, sq, h, d), 7.0, device="cuda", dtype=torch.bfloat16)
    lse = torch.full((b, h, sq), 7.0, device="cuda")
    qd, kd, vd = qq.cuda(), kk.cuda(), vv.cuda()
    lib.fmha_fwd_fp8(qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), lse.data_ptr(),
                          qs, ks, vs, sq, sk, b, h, hk, d, d ** -0.5, -1, 0 if causal else -1, False,
                          capi.stream_handle())
    torch.cuda.synchronize()
    assert lib.fmha_last_status() == 0, lib.fmha_last_error()
    ro, rl = ref_attn(qq.float() * qs, kk.float() * ks, vv.float() * vs, causal)
    o = out.float().cpu()
    l = lse.cpu()
    nan = torch.isnan(o)
    err = (o - ro).abs()
    err[nan] = float("inf")
    print(f"== {name}: b{b} sq{sq} sk{sk} h{h}/{hk} causal={causal}")
    print(f"   nan {int(nan.sum())}/{o.numel()}  max err(finite) {err[~nan].max().item() if (~nan).any() else -1:.4g}"
          f"  ref max {ro.abs().max().item():.3g}  lse err {(l - rl).abs().nan_to_num(1e9).max().item():.4g}"
          f"  lse nan {int(torch.isnan(l).sum())}")
    bad = err > 0.05 + 0.05 * ro.abs()
    if bad.any():
        idx = bad.nonzero()
        rows = idx[:, 1] * 0 + idx[:, 1]                  # query position
        # row within the item (G = h / hk rows per position)
        G = h // hk
        row = idx[:, 1] * G + (idx[:, 2] % G)
        print(f"   bad {int(bad.sum())}: item-row%256 hist (by wave):",
              torch.bincount((row % 256) // 64, minlength=4).tolist(),
              " rb:", torch.bincount((row % 64) // 32, minlength=2).tolist(),
              " lane-row%32 (first 32):", torch.bincount(row % 32, minlength=32).tolist())
        print("   d%32 hist:", torch.bincount(idx[:, 3] % 32, minlength=32).tolist(),
              " d//32:", torch.bincount(idx[:, 3] // 32, minlength=4).tolist(),
              " pos range:", int(rows.min()), int(rows.max()))
        i0 = idx[0].tolist()
        print(f"   first bad at {i0}: got {o[tuple(i0)].item():.4g} want {ro[tuple(i0)].item():.4g}")
        # relation: got vs ref along d at that row
        bb, s_, hh = i0[:3]
        print("   row got :", [round(x, 3) for x in o[bb, s_, hh, :8].tolist()])
        print("   row want:", [round(x, 3) for x in ro[bb, s_, hh, :8].tolist()])


def main():
    from xf_flash_attention_cutlass_amd import capi
    lib = capi.lib()
    assert lib.fmha_set_option(b"fp8_w4", 1) == 0
    g = torch.Generator().manual_seed(0)
    R = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    d = 128
    # 1) one item, one tile, everything visible
    for sq, sk in ((256, 64), (256, 128), (256, 256), (256, 320), (300, 300), (256, 1024)):
        run(lib, "random", R(1, sq, 1, d), R(1, sk, 1, d), R(1, sk, 1, d), False)
    # 2) Q = 0: uniform P, O = mean of V (PV path only)
    run(lib, "q0", torch.zeros(1, 256, 1, d), R(1, 256, 1, d), R(1, 256, 1, d), False)
    # 3) V = one-hot along d per key (v[key, d] = 1 iff d == key % 128): O[row, d] = P mass
    v = torch.zeros(1, 256, 1, d)
    v[0, torch.arange(256), 0, torch.arange(256) % d] = 1.0
    run(lib, "vonehot", R(1, 256, 1, d), R(1, 256, 1, d), v, False)
    # 4) V = 1: O = 1 (normalisation)
    run(lib, "v1", R(1, 256, 1, d), R(1, 256, 1, d), torch.ones(1, 256, 1, d), False)
    # 5) causal, GQA
    run(lib, "causal", R(1, 512, 4, d), R(1, 512, 2, d), R(1, 512, 2, d), True)
    run(lib, "bigger", R(2, 1024, 8, d), R(2, 1024, 2, d), R(2, 1024, 2, d), False)


if __name__ == "__main__":
    main()

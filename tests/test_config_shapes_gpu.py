"""GPU parity at the BASELINE configurations' full shapes (the shapes bench.py times).

Each test runs the HIP path at exactly the benched shape, then checks sampled (batch, head) /
sequence slices against the pinned CPU oracle with the reference's own rules (test.py:975 fwd,
:984-986 gradients, :1593-1594 kvcache; LSE within 1e-3), and covers the rest of the output
with size-independent properties (bitwise equality with another schedule of the same kernel).
LSE gate: 1e-3 absolute (fp32 intermediates).
Per-case max|err| and the bound are collected into the parity report (XFA_PARITY_REPORT).

  C2  mha_fwd  B4 H32 S4096 D128 bf16 causal (persistent XCD-paired schedule, 512 items)
  C3  mha_fwd + mha_bwd, same shape
  C4  mha_varlen_fwd, bench.varlen_lengths(): 32 ragged sequences, 131072 tokens, H32 D128
  C5  paged decode B8 H32 Hk8 Sq1, cache 32768, page 16, fp8 e4m3fn K/V, random-permutation
      block table, the 32-split decode path
"""
import pytest
import torch

import bench
from oracle import attention_ref as orc
from tests import test_fwd4_redo_gpu as r4

pytestmark = pytest.mark.gpu
DEV = "cuda"
LSE_ATOL = 1e-3
LSE_ATOL_DEC = 1e-3


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


def _lib():
    from xf_flash_attention_cutlass_amd import capi
    return capi.lib()


def _check(report, case, got, ref, pt, mult, atol=0.0):
    ok, err, bound = orc.parity_ok(got.cpu(), ref, pt, mult, atol)
    report({"case": case, "err": err, "bound": bound, "mult": mult, "ok": bool(ok)})
    assert ok, f"{case}: max|out-ref|={err:.3g} > bound {bound:.3g}"


def _rand(shape, seed, dtype=torch.bfloat16):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, device=DEV, dtype=dtype, generator=g)


SAMPLE_BH = [(0, 0), (1, 17), (2, 9), (3, 31)]     # every batch of B = 4


def test_c2_full_shape(xfa, parity_report):
    B, S, H, D = 4, 4096, 32, 128
    q, k, v = _rand((B, S, H, D), 1), _rand((B, S, H, D), 2), _rand((B, S, H, D), 3)
    out, lse, _ = xfa.flash_attn_func(q, k, v, causal=True, return_attn_probs=True)
    torch.cuda.synchronize()
    assert _lib().fmha_last_num_splits() == 1
    kern = _lib().fmha_last_kernel().decode()
    want = r4.expected_kernel(_lib().fmha_get_option(b"fwd_w4"), 0)     # causal
    assert kern.startswith(want + " "), kern
    for b, h in SAMPLE_BH:
        qs, ks, vs = (x[b:b + 1, :, h:h + 1].cpu() for x in (q, k, v))
        ref, _ = orc.attention_ref(qs, ks, vs, causal=True)
        pt, _ = orc.attention_ref(qs, ks, vs, causal=True, upcast=False, reorder_ops=True)
        _check(parity_report, f"C2 out b{b} h{h}", out[b:b + 1, :, h:h + 1], ref, pt, 2.0)
        lref = orc.attention_lse_ref(qs, ks, causal=True)
        lerr = (lse[b:b + 1, h:h + 1].cpu() - lref).abs().max().item()
        parity_report({"case": f"C2 lse b{b} h{h}", "err": lerr, "bound": LSE_ATOL,
                       "ok": lerr < LSE_ATOL})
        assert lerr < LSE_ATOL
    # every head: the persistent schedule == one workgroup per item, bit for bit
    L = _lib()
    assert L.fmha_set_option(b"fwd_persistent", 0) == 0
    try:
        out_np = xfa.flash_attn_func(q, k, v, causal=True)
    finally:
        L.fmha_set_option(b"fwd_persistent", 1)
    assert torch.equal(out, out_np)
    # ... == the per-XCD dynamic item queues (fwd_dyn = 2), twice (self-resetting counters)
    dyn = L.fmha_get_option(b"fwd_dyn")
    assert L.fmha_set_option(b"fwd_dyn", 2) == 0
    try:
        for _ in range(2):
            out_dyn = xfa.flash_attn_func(q, k, v, causal=True)
            assert torch.equal(out, out_dyn)
    finally:
        L.fmha_set_option(b"fwd_dyn", dyn)


def test_c3_full_shape(xfa, parity_report):
    B, S, H, D = 4, 4096, 32, 128
    q, k, v, g = (_rand((B, S, H, D), s) for s in (4, 5, 6, 7))
    qd, kd, vd = (x.clone().requires_grad_(True) for x in (q, k, v))
    out = xfa.flash_attn_func(qd, kd, vd, causal=True)
    dq, dk, dv = torch.autograd.grad(out, (qd, kd, vd), g)
    torch.cuda.synchronize()
    for b, h in SAMPLE_BH:
        sl = [x[b:b + 1, :, h:h + 1].cpu() for x in (q, k, v, g)]
        grads = []
        for up in (True, False):
            qq, kk, vv = (x.clone().requires_grad_(True) for x in sl[:3])
            o, _ = orc.attention_ref(qq, kk, vv, causal=True, upcast=up, reorder_ops=not up)
            grads.append(torch.autograd.grad(o, (qq, kk, vv), sl[3]))
        for nm, got, r, p in zip(("dq", "dk", "dv"), (dq, dk, dv), *grads):
            _check(parity_report, f"C3 {nm} b{b} h{h}", got[b:b + 1, :, h:h + 1], r, p, 3.0, 1e-5)
    # deterministic mode at the full shape: bitwise reproducible, dK/dV identical
    qd2, kd2, vd2 = (x.clone().requires_grad_(True) for x in (q, k, v))
    out2 = xfa.flash_attn_func(qd2, kd2, vd2, causal=True, deterministic=True)
    d2 = torch.autograd.grad(out2, (qd2, kd2, vd2), g)
    assert torch.equal(d2[1], dk) and torch.equal(d2[2], dv)
    err = (d2[0].float() - dq.float()).abs().max().item()
    parity_report({"case": "C3 dq deterministic vs atomic", "err": err, "bound": 2e-2,
                   "ok": err < 2e-2})
    assert err < 2e-2


def test_c4_full_shape(xfa, parity_report):
    lens = bench.varlen_lengths()
    assert len(lens) == 32 and sum(lens) == 131072
    H, D = 32, 128
    tot = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    q, k, v = (_rand((tot, H, D), s) for s in (8, 9, 10))
    out, lse, _ = xfa.flash_attn_varlen_func(q, k, v, cu.to(DEV), cu.to(DEV), max(lens),
                                             max(lens), causal=True, return_attn_probs=True)
    torch.cuda.synchronize()
    for i, h in ((0, 0), (11, 5), (20, 16), (31, 31)):
        a, b = int(cu[i]), int(cu[i + 1])
        qs, ks, vs = (x[a:b, h:h + 1][None].cpu() for x in (q, k, v))
        ref, _ = orc.attention_ref(qs, ks, vs, causal=True)
        pt, _ = orc.attention_ref(qs, ks, vs, causal=True, upcast=False, reorder_ops=True)
        _check(parity_report, f"C4 out seq{i} (len {b - a}) h{h}", out[a:b, h:h + 1][None], ref,
               pt, 2.0)
        lref = orc.attention_lse_ref(qs, ks, causal=True)[0, 0]
        lerr = (lse[h, a:b].cpu() - lref).abs().max().item()
        parity_report({"case": f"C4 lse seq{i} h{h}", "err": lerr, "bound": LSE_ATOL,
                       "ok": lerr < LSE_ATOL})
        assert lerr < LSE_ATOL
    # every sequence and head: the per-XCD dynamic queues == the static schedule, bit for bit
    L = _lib()
    assert L.fmha_set_option(b"fwd_dyn", 0) == 0
    try:
        out_static = xfa.flash_attn_varlen_func(q, k, v, cu.to(DEV), cu.to(DEV), max(lens),
                                                max(lens), causal=True)
    finally:
        L.fmha_set_option(b"fwd_dyn", 1)
    assert torch.equal(out, out_static)


@pytest.mark.parametrize("ragged", [False, True])
def test_c5_full_shape(xfa, parity_report, ragged):
    """The benched decode shape and path: B8 H32 Hk8, 32768 cached tokens per sequence, page 16,
    fp8 e4m3fn K/V (scales 1/16), random-permutation block table; the split heuristic picks the
    32-split decode launch (checked).  ragged: the cache lengths of `bench.py --ragged`
    (U[1, 32768], the same generator seed).  Every sequence is compared with the oracle over the
    dequantised cache (kvcache rule, test.py:1593-1594)."""
    B, S, H, HK, D, page = 8, 32768, 32, 8, 128, 16
    nblk = S // page
    nblocks = B * nblk
    table = torch.randperm(nblocks, generator=torch.Generator().manual_seed(0)).to(torch.int32)
    table = table.view(B, nblk)
    ks, vs = 1.0 / 16, 1.0 / 16
    kc8 = (_rand((nblocks, page, HK, D), 11).float() / ks).to(torch.float8_e4m3fn)
    vc8 = (_rand((nblocks, page, HK, D), 12).float() / vs).to(torch.float8_e4m3fn)
    q = _rand((B, 1, H, D), 13)
    if ragged:
        lens = torch.randint(1, S + 1, (B,), generator=torch.Generator().manual_seed(0))
    else:
        lens = torch.full((B,), S)
    seqlens = lens.to(torch.int32).to(DEV)
    out, lse = xfa.flash_attn_with_kvcache(q, kc8, vc8, cache_seqlens=seqlens,
                                           block_table=table.to(DEV), k_scale=ks, v_scale=vs,
                                           return_softmax_lse=True)
    torch.cuda.synchronize()
    assert _lib().fmha_last_num_splits() == 32
    idx = table.long().to(DEV)
    k8u, v8u = kc8.view(torch.uint8), vc8.view(torch.uint8)
    for b in range(B):
        # gather this sequence's pages (as bytes), dequantise exactly: f32(fp8) * 2^-4 -> bf16
        kd = (k8u[idx[b]].view(torch.float8_e4m3fn).float() * ks).bfloat16()
        vd = (v8u[idx[b]].view(torch.float8_e4m3fn).float() * vs).bfloat16()
        n = int(lens[b])
        kd, vd = kd.reshape(1, S, HK, D)[:, :n].cpu(), vd.reshape(1, S, HK, D)[:, :n].cpu()
        qs = q[b:b + 1].cpu()
        ref, _ = orc.attention_ref(qs, kd, vd)
        pt, _ = orc.attention_ref(qs, kd, vd, upcast=False, reorder_ops=True)
        tag = f"C5{' ragged' if ragged else ''} b{b} len{n}"
        _check(parity_report, f"{tag} out", out[b:b + 1], ref, pt, 3.0, 1e-5)
        lref = orc.attention_lse_ref(qs, kd)
        lerr = (lse[b:b + 1].cpu() - lref).abs().max().item()
        parity_report({"case": f"{tag} lse", "err": lerr, "bound": LSE_ATOL_DEC,
                       "ok": lerr < LSE_ATOL_DEC})
        assert lerr < LSE_ATOL_DEC

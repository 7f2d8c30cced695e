"""GPU: the LSE the build returns under causal ALiBi follows the reference kernel's convention.

The reference kernel biases a causal score by `+slope * col` (mask_hip.h:163-164), its
non-causal form is `-slope * |row + sk - sq - col|` (:165-166).  The build's kernels use the
second form for causal rows too (its maximum, 0, sits on the diagonal, which their in-loop
reference max needs), and turn the LSE into the reference's convention afterwards (the two
differ by the row constant slope * (pos + sk - sq): O is the same, the LSE is not).  The
backward converts it back before reading it.  LSE within 1e-3 of the fp32 log-sum-exp of the
kernel-form scores (oracle.alibi_bias_kernel); O and gradients by the reference's rules
(test.py:975, 984-986).
"""
import pytest
import torch

from oracle import attention_ref as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"
LSE_ATOL = 1e-3


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


def _lse_close(lse, lse_ref, what):
    lse, lse_ref = lse.float().cpu(), lse_ref.float()
    fin = torch.isfinite(lse_ref)
    assert torch.equal(torch.isinf(lse), ~fin), what
    err = (lse[fin] - lse_ref[fin]).abs().max().item()
    assert err < LSE_ATOL, f"{what}: max|lse - ref| = {err:.3g}"


@pytest.mark.parametrize("sq,sk,h,hk,d", [(300, 300, 4, 4, 128), (200, 517, 4, 2, 64),
                                          (517, 200, 2, 1, 128), (129, 300, 2, 2, 256)])
def test_causal_alibi_lse_dense(xfa, sq, sk, h, hk, d):
    g = torch.Generator().manual_seed(sq + sk)
    b = 2
    q = torch.randn(b, sq, h, d, generator=g).bfloat16()
    k = torch.randn(b, sk, hk, d, generator=g).bfloat16()
    v = torch.randn(b, sk, hk, d, generator=g).bfloat16()
    slopes = torch.rand(b, h, generator=g) * 0.5
    out, lse, _ = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=True,
                                      alibi_slopes=slopes.to(DEV), return_attn_probs=True)
    bias_o = orc.alibi_bias(slopes, sq, sk, causal=True)     # test.py's form: same O
    ref, _ = orc.attention_ref(q, k, v, attn_bias=bias_o, causal=True)
    pt, _ = orc.attention_ref(q, k, v, attn_bias=bias_o, causal=True, upcast=False, reorder_ops=True)
    ok, err, bound = orc.parity_ok(out.float().cpu(), ref, pt, 2.0, 1e-5)
    assert ok, f"O: {err:.3g} > {bound:.3g}"
    lref = orc.attention_lse_ref(q, k, attn_bias=orc.alibi_bias_kernel(slopes, sq, sk, causal=True),
                                 causal=True)
    _lse_close(lse, lref, f"dense causal alibi {sq}x{sk} d{d}")


def test_causal_alibi_lse_varlen(xfa):
    g = torch.Generator().manual_seed(7)
    lens_q, lens_k = [100, 1, 333, 64], [150, 40, 333, 10]
    h, d = 4, 128
    cq = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
    ck = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
    q = torch.randn(int(cq[-1]), h, d, generator=g).bfloat16()
    k = torch.randn(int(ck[-1]), h, d, generator=g).bfloat16()
    v = torch.randn(int(ck[-1]), h, d, generator=g).bfloat16()
    slopes = torch.rand(len(lens_q), h, generator=g) * 0.5
    out, lse, _ = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cq.to(DEV), ck.to(DEV),
                                             max(lens_q), max(lens_k), causal=True,
                                             alibi_slopes=slopes.to(DEV), return_attn_probs=True)
    lse = lse.cpu()                                  # [h, total_q]
    for i in range(len(lens_q)):
        a, b = int(cq[i]), int(cq[i + 1])
        c, e = int(ck[i]), int(ck[i + 1])
        s = slopes[i:i + 1]
        lref = orc.attention_lse_ref(q[a:b][None], k[c:e][None],
                                     attn_bias=orc.alibi_bias_kernel(s, b - a, e - c, causal=True),
                                     causal=True)[0]
        _lse_close(lse[:, a:b], lref, f"varlen seq {i}")


@pytest.mark.parametrize("num_splits", [1, 4])
def test_causal_alibi_lse_paged_decode(xfa, num_splits):
    """paged decode (Sq = 1) and a split-KV combine: the LSE pass runs on the final LSE"""
    g = torch.Generator().manual_seed(11)
    b, h, hk, d, page, sk = 3, 8, 2, 128, 16, 300
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    q = torch.randn(b, 1, h, d, generator=g).bfloat16()
    lens = torch.tensor([300, 17, 129], dtype=torch.int32)
    slopes = torch.rand(b, h, generator=g) * 0.5
    out, lse = xfa.flash_attn_with_kvcache(q.to(DEV), kp.to(DEV), vp.to(DEV), cache_seqlens=lens.to(DEV),
                                           block_table=table.to(DEV), causal=True,
                                           alibi_slopes=slopes.to(DEV), num_splits=num_splits,
                                           return_softmax_lse=True)
    lse = lse.cpu()
    for i in range(b):
        n = int(lens[i])
        kk = kp[table[i].long()].reshape(1, -1, hk, d)[:, :n]
        lref = orc.attention_lse_ref(q[i:i + 1], kk,
                                     attn_bias=orc.alibi_bias_kernel(slopes[i:i + 1], 1, n, causal=True),
                                     causal=True)
        _lse_close(lse[i:i + 1], lref, f"decode seq {i} splits {num_splits}")


@pytest.mark.parametrize("deterministic", [False, True])
def test_causal_alibi_bwd_reads_converted_lse(xfa, deterministic):
    """the backward is handed the reference-convention LSE and must convert it back: its
    gradients against oracle autograd (3x + 1e-5, test.py:984-986)"""
    g = torch.Generator().manual_seed(5)
    b, s, h, d = 2, 300, 4, 128
    q = (torch.randn(b, s, h, d, generator=g) * 2).bfloat16()
    k, v, do = (torch.randn(b, s, h, d, generator=g).bfloat16() for _ in range(3))
    slopes = torch.rand(b, h, generator=g) * 0.5
    qd, kd, vd = (x.to(DEV).requires_grad_(True) for x in (q, k, v))
    out = xfa.flash_attn_func(qd, kd, vd, causal=True, alibi_slopes=slopes.to(DEV),
                              deterministic=deterministic)
    got = torch.autograd.grad(out, (qd, kd, vd), do.to(DEV))
    bias = orc.alibi_bias(slopes, s, s, causal=True)
    for up, dst in ((True, "ref"), (False, "pt")):
        qq, kk, vv = (x.clone().requires_grad_(True) for x in (q, k, v))
        o, _ = orc.attention_ref(qq, kk, vv, attn_bias=bias, causal=True, upcast=up, reorder_ops=not up)
        if up:
            ref = torch.autograd.grad(o, (qq, kk, vv), do)
        else:
            pt = torch.autograd.grad(o, (qq, kk, vv), do)
    for nm, x, r, p in zip(("dq", "dk", "dv"), got, ref, pt):
        ok, err, bound = orc.parity_ok(x.cpu(), r, p, 3.0, 1e-5)
        assert ok, f"{nm}: {err:.3g} > {bound:.3g}"


def test_causal_alibi_long_linear_frame(xfa):
    """The ping-pong kernel runs causal ALiBi in the linear frame (bias slope * key, the tile base
    folded into the subtracted max, gen_fwdpp.py _alibi_linear_ops): at 8192 keys and the largest
    slope (0.5) the frame's offsets reach 4096 in score units, so O and the LSE are checked there,
    the LSE against the fp32 log-sum-exp with 4 fp32 ulps of its magnitude added to LSE_ATOL (the
    reference-convention LSE is itself of that size).  One varlen sequence: a single pass, as the
    reference forces for varlen (no split-KV heuristic at two heads)."""
    from xf_flash_attention_cutlass_amd import capi
    g = torch.Generator().manual_seed(8192)
    s, h, d = 8192, 2, 128
    q = torch.randn(s, h, d, generator=g).bfloat16()
    k = torch.randn(s, h, d, generator=g).bfloat16()
    v = torch.randn(s, h, d, generator=g).bfloat16()
    cu = torch.tensor([0, s], dtype=torch.int32)
    slopes = torch.tensor([[0.5, 2.0 ** -7]])
    out, lse, _ = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cu.to(DEV), cu.to(DEV),
                                             s, s, causal=True, alibi_slopes=slopes.to(DEV),
                                             return_attn_probs=True)
    kern = capi.lib().fmha_last_kernel().decode()
    assert kern.startswith("fmha_fwdpp_kernel "), kern
    bias_o = orc.alibi_bias(slopes, s, s, causal=True)
    ref, _ = orc.attention_ref(q[None], k[None], v[None], attn_bias=bias_o, causal=True)
    pt, _ = orc.attention_ref(q[None], k[None], v[None], attn_bias=bias_o, causal=True, upcast=False,
                              reorder_ops=True)
    ok, err, bound = orc.parity_ok(out[None].float().cpu(), ref, pt, 2.0, 1e-5)
    assert ok, f"O: {err:.3g} > {bound:.3g}"
    lref = orc.attention_lse_ref(q[None], k[None], attn_bias=orc.alibi_bias_kernel(slopes, s, s, causal=True),
                                 causal=True)[0].float()
    lse = lse.float().cpu()                          # [h, total_q]
    tol = LSE_ATOL + 4 * torch.finfo(torch.float32).eps * lref.abs()
    err = (lse - lref).abs()
    assert bool((err <= tol).all()), f"max|lse - ref| = {err.max().item():.3g}, tol {tol.max().item():.3g}"

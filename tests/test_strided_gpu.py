"""GPU parity of non-dense inputs: head- and batch-sliced views, kv-packed and qkv-packed
tensors, and views at storage offsets that are not 16-byte aligned.

`paged_attn.fwd` hands 16-byte-aligned views with d % 8 == 0 to `fmha_fwd_strided` without a copy
(q_row != h * d, k_row != hk * d, the 4-wave kernel's k_row == v_row case of kv-packed inputs);
anything else is copied to an aligned contiguous tensor first.  Forward and backward are checked
against the oracle on contiguous CPU copies of sampled (batch, head) slices, with the reference's
rules (test.py:975 fwd 2x, :984-986 gradients 3x + 1e-5).
"""
import pytest
import torch

from oracle import attention_ref as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


def _check(what, got, ref, pt, mult, atol=0.0):
    ok, err, bound = orc.parity_ok(got.cpu(), ref, pt, mult, atol)
    assert ok, f"{what}: max|got-ref|={err:.3g} > bound {bound:.3g}"


def _run(xfa, q, k, v, g, causal, kvpacked=None):
    """fwd + bwd on the given (possibly strided) leaves; returns out and the leaves' grads."""
    if kvpacked is not None:
        out = xfa.flash_attn_kvpacked_func(q, kvpacked, causal=causal)
        dq, dkv = torch.autograd.grad(out, (q, kvpacked), g)
        return out, dq, dkv[:, :, 0], dkv[:, :, 1]
    out = xfa.flash_attn_func(q, k, v, causal=causal)
    return (out, *torch.autograd.grad(out, (q, k, v), g))


def _oracle_check(tag, q, k, v, g, out, dq, dk, dv, causal, samples):
    G = q.shape[2] // k.shape[2]
    for b, h in samples:
        kh = h // G
        qs, gs = (x[b:b + 1, :, h:h + 1].detach().cpu().contiguous() for x in (q, g))
        ks, vs = (x[b:b + 1, :, kh:kh + 1].detach().cpu().contiguous() for x in (k, v))
        res = []
        for up in (True, False):
            qq, kk, vv = (x.clone().requires_grad_(True) for x in (qs, ks, vs))
            o, _ = orc.attention_ref(qq, kk, vv, causal=causal, upcast=up, reorder_ops=not up)
            res.append((o, *torch.autograd.grad(o, (qq, kk, vv), gs)))
        (o_ref, *g_ref), (o_pt, *g_pt) = res
        _check(f"{tag} out b{b} h{h}", out[b:b + 1, :, h:h + 1], o_ref, o_pt, 2.0)
        _check(f"{tag} dq b{b} h{h}", dq[b:b + 1, :, h:h + 1], g_ref[0], g_pt[0], 3.0, 1e-5)
        if G == 1:   # dK / dV of a kv head sum over its G query heads
            _check(f"{tag} dk b{b} h{h}", dk[b:b + 1, :, kh:kh + 1], g_ref[1], g_pt[1], 3.0, 1e-5)
            _check(f"{tag} dv b{b} h{h}", dv[b:b + 1, :, kh:kh + 1], g_ref[2], g_pt[2], 3.0, 1e-5)


def _randn(shape, seed, dtype):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, device=DEV, generator=g).to(dtype)


CASES = [  # b, s, h, hk, d  (the d128 bf16 cases are large enough for one pass / the 4-wave kernel)
    (2, 300, 4, 2, 64),
    (2, 517, 4, 4, 64),
    (4, 2048, 16, 8, 128),
    (2, 333, 6, 2, 128),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("b,s,h,hk,d", CASES)
def test_head_and_batch_sliced_views(xfa, dtype, causal, b, s, h, hk, d):
    """q, k, v are head slices of wider tensors and batch slices of longer ones (k and v with
    the same row stride, as the 4-wave kernel's shared DMA offsets need: the same kernel runs as
    for the contiguous copies, so the bytes must agree)."""
    qf = _randn((b + 2, s, h + 3, d), 1, dtype)
    kf = _randn((b + 2, s, hk + 2, d), 2, dtype)
    vf = _randn((b + 2, s, hk + 2, d), 3, dtype)
    q = qf[1:b + 1, :, 2:h + 2].detach().requires_grad_(True)
    k = kf[2:b + 2, :, 1:hk + 1].detach().requires_grad_(True)
    v = vf[0:b, :, 1:hk + 1].detach().requires_grad_(True)
    assert not q.is_contiguous() and not k.is_contiguous() and not v.is_contiguous()
    g = _randn((b, s, h, d), 4, dtype)
    out, dq, dk, dv = _run(xfa, q, k, v, g, causal)
    # the same call on contiguous copies gives the same bytes (the strides only address)
    qc, kc, vc = (x.detach().contiguous().requires_grad_(True) for x in (q, k, v))
    out_c, dq_c, dk_c, dv_c = _run(xfa, qc, kc, vc, g, causal)
    assert torch.equal(out, out_c) and torch.equal(dk, dk_c) and torch.equal(dv, dv_c)
    assert (dq.float() - dq_c.float()).abs().max().item() < 2e-2     # dQ atomics' order
    _oracle_check(f"sliced {b}x{s} h{h}/{hk} d{d} c{causal}", q, k, v, g, out, dq, dk, dv,
                  causal, ((0, 0), (b - 1, h - 1)))


@pytest.mark.parametrize("b,s,h,hk,d", CASES)
def test_sliced_views_k_v_row_strides_differ(xfa, b, s, h, hk, d):
    """k and v slices of tensors with different head counts (k_row != v_row): the 8-wave
    kernel's path; against the oracle."""
    dtype = torch.bfloat16
    q = _randn((b, s, h + 1, d), 21, dtype)[:, :, 1:].detach().requires_grad_(True)
    k = _randn((b, s, hk + 3, d), 22, dtype)[:, :, :hk].detach().requires_grad_(True)
    v = _randn((b, s, hk + 1, d), 23, dtype)[:, :, 1:].detach().requires_grad_(True)
    g = _randn((b, s, h, d), 24, dtype)
    out, dq, dk, dv = _run(xfa, q, k, v, g, True)
    _oracle_check(f"k/v strides differ {b}x{s} h{h}/{hk} d{d}", q, k, v, g, out, dq, dk, dv,
                  True, ((0, 0), (b - 1, h - 1)))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("b,s,h,hk,d", CASES)
def test_kvpacked(xfa, dtype, b, s, h, hk, d):
    """kv [b, s, 2, hk, d]: k = kv[:, :, 0], v = kv[:, :, 1] (k_row = v_row = 2 hk d)."""
    q = _randn((b, s, h, d), 5, dtype).requires_grad_(True)
    kv = _randn((b, s, 2, hk, d), 6, dtype).requires_grad_(True)
    g = _randn((b, s, h, d), 7, dtype)
    out, dq, dk, dv = _run(xfa, q, None, None, g, True, kvpacked=kv)
    _oracle_check(f"kvpacked {b}x{s} h{h}/{hk} d{d}", q, kv[:, :, 0], kv[:, :, 1], g, out, dq,
                  dk, dv, True, ((0, 0), (b - 1, h - 1)))


@pytest.mark.parametrize("d", [64, 128])
def test_qkv_packed_views(xfa, d):
    """q, k, v = qkv[:, :, 0..2] of one [b, s, 3, h, d] tensor (q_row = 3 h d)."""
    b, s, h = 4, 2048 if d == 128 else 400, 16
    qkv = _randn((b, s, 3, h, d), 8, torch.bfloat16).requires_grad_(True)
    g = _randn((b, s, h, d), 9, torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    out = xfa.flash_attn_func(q, k, v, causal=True)
    (dqkv,) = torch.autograd.grad(out, (qkv,), g)
    _oracle_check(f"qkv-packed d{d}", q, k, v, g, out, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
                  True, ((0, 0), (b - 1, h - 1)))


@pytest.mark.parametrize("d", [64, 128])
def test_misaligned_views(xfa, d):
    """Contiguous views starting 2 bytes past a 16-byte boundary: copied to aligned tensors by
    the binding (the kernels' 16-byte loads need aligned bases), same bytes as aligned inputs."""
    b, s, h = 2, 300, 4
    n = b * s * h * d
    outs = []
    for off in (0, 1):
        bufs = [torch.zeros(n + 8, device=DEV, dtype=torch.bfloat16) for _ in range(3)]
        for i, buf in enumerate(bufs):
            buf[off:off + n] = _randn((n,), 10 + i, torch.bfloat16)
        q, k, v = (buf[off:off + n].view(b, s, h, d) for buf in bufs)
        if off:
            assert q.data_ptr() % 16 == 2
        outs.append(xfa.flash_attn_func(q, k, v, causal=True))
    assert torch.equal(outs[0], outs[1])

"""GPU parity: the gfx950 forward kernels vs the reference oracle.

Pass rule = the reference's own (test.py:975, 1296, 1593-1594): max|out - out_ref| must be at
most 2x (fwd, varlen) or 3x + 1e-5 (kvcache) the error of the low-precision PyTorch path
max|out_pt - out_ref|.  LSE (fp32) is checked against the fp32 log-sum-exp of the oracle
(oracle.attention_lse_ref) with an absolute tolerance of 1e-3 (fp32 intermediates
within 1e-3; the kernels sum the fp32 P as the reference's softmax does).
"""
import math

import pytest
import torch

from oracle import attention_ref as orc
from tests import golden_util as gu

pytestmark = pytest.mark.gpu
DEV = "cuda"
LSE_ATOL = 1e-3


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


def _dtype(name):
    return {"float16": torch.float16, "bfloat16": torch.bfloat16}[name]


def _assert_parity(out, out_ref, out_pt, mult=2.0, atol=0.0, what=""):
    ok, err, bound = orc.parity_ok(out.cpu(), out_ref, out_pt, mult, atol)
    assert ok, f"{what}: max|out-ref|={err:.3g} > bound {bound:.3g}"


@pytest.mark.parametrize("name", [n for n in gu.names("fwd") if "fp32" not in n])
def test_fwd_golden(xfa, name):
    t, m = gu.load(name)
    q, k, v = (t[x].to(DEV) for x in ("q", "k", "v"))
    slopes = t["alibi_slopes"].to(DEV) if m["alibi"] else None
    out, lse, _ = xfa.flash_attn_func(q, k, v, 0.0, causal=m["causal"],
                                      window_size=tuple(m["window"]), softcap=m["softcap"],
                                      alibi_slopes=slopes, return_attn_probs=True)
    torch.cuda.synchronize()
    _assert_parity(out, t["out_ref"], t["out_pt"], what=name)
    bias = None
    if m["alibi"]:   # the reference kernel's ALiBi form (causal: +slope*col, mask_hip.h:163-164)
        bias = orc.alibi_bias_kernel(t["alibi_slopes"], m["sq"], m["sk"], causal=m["causal"])
    lse_ref = orc.attention_lse_ref(t["q"], t["k"], attn_bias=bias, causal=m["causal"],
                                    window_size=tuple(m["window"]), softcap=m["softcap"])
    fin = torch.isfinite(lse_ref)
    assert torch.equal(torch.isinf(lse.cpu()), ~fin)
    assert (lse.cpu()[fin] - lse_ref[fin]).abs().max().item() < LSE_ATOL


def oracle_window(window, sk):
    """API windows use -1 for 'unbounded'; the oracle's local branch (test.py:300-307) reads a
    negative right window literally once the left one is set, so spell it out as sk there."""
    wl, wr = window
    return (wl, sk) if (wl >= 0 and wr < 0) else (wl, wr)


def _rand_case(b, h, hk, sq, sk, d, dtype, causal, window=(-1, -1), seed=0):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(b, sq, h, d, generator=g).to(dtype)
    k = torch.randn(b, sk, hk, d, generator=g).to(dtype)
    v = torch.randn(b, sk, hk, d, generator=g).to(dtype)
    w = oracle_window(window, sk)
    out_ref, _ = orc.attention_ref(q, k, v, causal=causal, window_size=w)
    out_pt, _ = orc.attention_ref(q, k, v, causal=causal, window_size=w, upcast=False,
                                  reorder_ops=True)
    return q, k, v, out_ref, out_pt


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("sq,sk,h,hk", [(1, 147, 4, 4), (113, 203, 4, 2), (128, 217, 2, 1),
                                        (512, 256, 2, 2), (1023, 1024, 2, 2), (2048, 2048, 1, 1),
                                        (300, 300, 6, 3)])
def test_fwd_random(xfa, dtype, causal, d, sq, sk, h, hk):
    q, k, v, out_ref, out_pt = _rand_case(1, h, hk, sq, sk, d, dtype, causal)
    out, lse, _ = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=causal,
                                      return_attn_probs=True)
    _assert_parity(out, out_ref, out_pt, what=f"{sq}x{sk} h{h}/{hk} d{d} c{causal}")
    lse_ref = orc.attention_lse_ref(q, k, causal=causal)
    fin = torch.isfinite(lse_ref)
    assert torch.equal(torch.isinf(lse.cpu()), ~fin)
    assert (lse.cpu()[fin] - lse_ref[fin]).abs().max().item() < LSE_ATOL


@pytest.mark.parametrize("window", [(0, 0), (17, 3), (100, -1), (-1, 40), (5, 200)])
def test_fwd_local_windows(xfa, window):
    q, k, v, out_ref, out_pt = _rand_case(2, 4, 2, 211, 333, 128, torch.bfloat16, False, window)
    out = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), window_size=window)
    _assert_parity(out, out_ref, out_pt, what=f"window {window}")


@pytest.mark.parametrize("d", [40, 80, 96, 104])
def test_fwd_padded_head_dims(xfa, d):
    q, k, v, out_ref, out_pt = _rand_case(2, 3, 3, 77, 190, d, torch.float16, True)
    out = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=True)
    assert out.shape == (2, 77, 3, d)
    _assert_parity(out, out_ref, out_pt, what=f"d={d}")


def test_fwd_alibi_softcap_combo(xfa):
    torch.manual_seed(3)
    b, h, sq, sk, d = 2, 4, 150, 150, 64
    q = (torch.randn(b, sq, h, d) * 5).half()
    k, v = torch.randn(b, sk, h, d).half(), torch.randn(b, sk, h, d).half()
    slopes = torch.rand(h) * 0.3
    bias = orc.alibi_bias(slopes.expand(b, h), sq, sk, causal=True)
    out_ref, _ = orc.attention_ref(q, k, v, attn_bias=bias, causal=True, softcap=30.0)
    out_pt, _ = orc.attention_ref(q, k, v, attn_bias=bias, causal=True, softcap=30.0,
                                  upcast=False, reorder_ops=True)
    out = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=True, softcap=30.0,
                              alibi_slopes=slopes.to(DEV))   # [H]-shaped slopes, B > 1
    _assert_parity(out, out_ref, out_pt, mult=5.0, what="alibi+softcap")


def test_fwd_capi_matches_pybind_bitwise(xfa):
    """The C ABI called directly (ctypes, no torch types) gives the pybind op's bytes."""
    from xf_flash_attention_cutlass_amd import capi
    q, k, v, _, _ = _rand_case(2, 8, 2, 257, 300, 128, torch.bfloat16, True)
    q, k, v = q.to(DEV), k.to(DEV), v.to(DEV)
    ref = xfa.flash_attn_func(q, k, v, causal=True)
    o = torch.empty_like(q)
    lse = torch.empty(2, 8, 257, device=DEV)
    L = capi.lib()
    L.fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, 257, 300, 2, 8, 2,
               128, 0.0, capi.stream_handle(), None, 128 ** -0.5, None, lse.data_ptr(), -1, 0,
               0.0, False, False, 0)
    capi.check()
    torch.cuda.synchronize()
    assert torch.equal(o, ref)


@pytest.mark.parametrize("splits", [2, 3, 7])
def test_fwd_split_kv_matches_single_pass(xfa, splits):
    from xf_flash_attention_cutlass_amd import capi
    q, k, v, out_ref, out_pt = _rand_case(1, 4, 4, 64, 1000, 128, torch.float16, False)
    q, k, v = q.to(DEV), k.to(DEV), v.to(DEV)
    outs = []
    for s in (1, splits):
        o = torch.empty_like(q)
        lse = torch.empty(1, 4, 64, device=DEV)
        capi.lib().fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, 64,
                            1000, 1, 4, 4, 128, 0.0, capi.stream_handle(), None, 128 ** -0.5,
                            None, lse.data_ptr(), -1, -1, 0.0, False, True, s)
        capi.check()
        outs.append((o, lse))
    torch.cuda.synchronize()
    _assert_parity(outs[1][0], out_ref, out_pt, what=f"splits={splits}")
    assert (outs[0][1] - outs[1][1]).abs().max().item() < 1e-4
    assert (outs[0][0].float() - outs[1][0].float()).abs().max().item() < 2e-3


def _assert_ulps(a, b, n, dtype, floor_rel=0.0):
    """|a - b| <= n ulps of dtype at max(|a|, |b|) elementwise (ulp = 2^(exponent - mantissa
    bits)), plus n x floor_rel x max|b| for elements near zero (an O element's fp32 sums carry the
    row's magnitude, not its own); infinities must match exactly"""
    a, b = a.float(), b.float()
    fin = torch.isfinite(b)
    assert torch.equal(fin, torch.isfinite(a)) and torch.equal(a[~fin], b[~fin])
    a, b = a[fin], b[fin]
    mant = {torch.bfloat16: 7, torch.float16: 10, torch.float32: 23}[dtype]
    _, e = torch.frexp(torch.maximum(a.abs(), b.abs()))
    ulp = torch.ldexp(torch.ones_like(a), e - 1 - mant)
    floor = floor_rel * b.abs().max().item()
    bad = (a - b).abs() > n * ulp + n * floor
    assert not bad.any(), (f"{int(bad.sum())} elements past {n} ulps: max diff "
                           f"{(a - b).abs().max().item():.3g}")


@pytest.mark.parametrize("d,splits,causal", [(64, 100, False), (128, 100, True), (256, 37, False),
                                             (128, 5, True)])
def test_split_combine_row_kernel(xfa, d, splits, causal):
    """The one-workgroup-per-row combine (comb_row=1, few rows) against the per-wave combine
    (comb_row=0) and the single pass: splits past the first 64-split batch of its loop, D = 64 /
    128 / 256, and causal rows that see no key of the last splits (empty partials, LSE -inf)."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(11)
    b, h, sq, sk = 1, 2, 40, 6500
    q = torch.randn(b, sq, h, d, dtype=torch.bfloat16, device=DEV)
    k = torch.randn(b, sk, h, d, dtype=torch.bfloat16, device=DEV)
    v = torch.randn(b, sk, h, d, dtype=torch.bfloat16, device=DEV)
    outs = {}
    for name, s, cr in (("single", 1, 1), ("row", splits, 1), ("wave", splits, 0)):
        assert L.fmha_set_option(b"comb_row", cr) == 0
        try:
            o = torch.empty_like(q)
            lse = torch.empty(b, h, sq, device=DEV)
            L.fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, sq, sk, b, h,
                       h, d, 0.0, capi.stream_handle(), None, d ** -0.5, None, lse.data_ptr(), -1,
                       0 if causal else -1, 0.0, False, False, s)
            capi.check()
            if s > 1:
                assert L.fmha_last_num_splits() == s
        finally:
            L.fmha_set_option(b"comb_row", 1)
        torch.cuda.synchronize()
        outs[name] = (o.float(), lse)
    (o1, l1), (o2, l2), (o3, l3) = outs["single"], outs["row"], outs["wave"]
    # the same fp32 partials, only reassociated: 2 bf16 ulps of O, 2 fp32 ulps of the LSE
    _assert_ulps(o2, o3, 2, torch.bfloat16, 2.0 ** -20)
    _assert_ulps(l2, l3, 2, torch.float32)
    assert (o2 - o1).abs().max().item() <= 2e-2
    assert (l2 - l1).abs().max().item() <= 1e-4


def test_fwd_sq_gt_sk_causal_empty_rows(xfa):
    """Bottom-right causal alignment: with sq > sk the first sq-sk rows see no key -> O = 0,
    LSE = +inf (flash_fwd_kernel_hip.h:626-670)."""
    q, k, v, out_ref, out_pt = _rand_case(1, 2, 2, 300, 100, 64, torch.bfloat16, True)
    out, lse, _ = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=True,
                                      return_attn_probs=True)
    assert (out[:, :200].float() == 0).all()
    assert torch.isinf(lse[:, :, :200]).all()
    _assert_parity(out, out_ref, out_pt, what="sq>sk causal")


def test_fwd_out_param_and_errors(xfa):
    q = torch.randn(1, 16, 2, 64, device=DEV, dtype=torch.float16)
    out = torch.empty_like(q)
    r = xfa.paged_attn.fwd(q, q, q, out, None, 0.0, 0.125, False, -1, -1, 0.0, False, None)
    assert r[0].data_ptr() == out.data_ptr()
    with pytest.raises(RuntimeError, match="fp16 and bf16"):
        xfa.paged_attn.fwd(q.float(), q.float(), q.float(), None, None, 0.0, 0.125, False, -1,
                           -1, 0.0, False, None)
    with pytest.raises(RuntimeError, match="must divide"):
        xfa.flash_attn_func(torch.randn(1, 16, 3, 64, device=DEV, dtype=torch.float16),
                            q, q)


# ----------------------------------------------------------------------------- varlen ----
@pytest.mark.parametrize("name", gu.names("varlen"))
def test_varlen_golden(xfa, name):
    t, m = gu.load(name)
    qpm, kpm = t["query_padding_mask"], t["key_padding_mask"]
    q_u, idx_q, cu_q, max_q = orc.unpad_input(t["q"], qpm)
    k_u, _, cu_k, max_k = orc.unpad_input(t["k"], kpm)
    v_u, _, _, _ = orc.unpad_input(t["v"], kpm)
    out_u, lse, _ = xfa.flash_attn_varlen_func(
        q_u.to(DEV), k_u.to(DEV), v_u.to(DEV), cu_q.to(DEV), cu_k.to(DEV), max_q, max_k,
        causal=m["causal"], window_size=tuple(m["window"]), return_attn_probs=True)
    out = orc.pad_input(out_u.cpu(), idx_q, m["b"], m["sq"])
    _assert_parity(out, t["out_ref"], t["out_pt"], what=name)
    assert lse.shape == (m["h"], q_u.shape[0])


def test_varlen_ragged_large(xfa):
    """Ragged lengths incl. 1-token and empty-key sequences; compared per sequence."""
    torch.manual_seed(0)
    h, hk, d = 4, 2, 128
    lq = [1, 300, 77, 1024, 5, 640]
    lk = [147, 300, 500, 1024, 1, 700]
    cu_q = torch.tensor([0] + list(torch.tensor(lq).cumsum(0)), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(lk).cumsum(0)), dtype=torch.int32)
    q = torch.randn(sum(lq), h, d).bfloat16()
    k = torch.randn(sum(lk), hk, d).bfloat16()
    v = torch.randn(sum(lk), hk, d).bfloat16()
    for causal in (False, True):
        out = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cu_q.to(DEV),
                                         cu_k.to(DEV), max(lq), max(lk), causal=causal).cpu()
        for i in range(len(lq)):
            qs = q[cu_q[i]:cu_q[i + 1]][None]
            ks, vs = k[cu_k[i]:cu_k[i + 1]][None], v[cu_k[i]:cu_k[i + 1]][None]
            r, _ = orc.attention_ref(qs, ks, vs, causal=causal)
            pt, _ = orc.attention_ref(qs, ks, vs, causal=causal, upcast=False, reorder_ops=True)
            _assert_parity(out[cu_q[i]:cu_q[i + 1]][None], r, pt, what=f"seq {i} c{causal}")


# ----------------------------------------------------------------------------- kvcache ---
@pytest.mark.parametrize("name", gu.names("kvcache"))
def test_kvcache_golden(xfa, name):
    t, m = gu.load(name)
    out = xfa.flash_attn_with_kvcache(
        t["q"].to(DEV), t["k_cache_paged"].to(DEV), t["v_cache_paged"].to(DEV),
        cache_seqlens=t["cache_seqlens"].to(DEV), block_table=t["block_table"].to(DEV),
        causal=m["causal"], window_size=tuple(m["window"]), num_splits=m["num_splits"])
    _assert_parity(out, t["out_ref"], t["out_pt"], mult=3.0, atol=1e-5, what=name)


@pytest.mark.parametrize("num_splits", [1, 0, 4])
@pytest.mark.parametrize("sq,hk", [(1, 8), (4, 2), (64, 4)])
def test_paged_indexing_bitexact(xfa, num_splits, sq, hk):
    """Paged O == O over the contiguous gather of the same pages, bit for bit."""
    torch.manual_seed(0)
    b, h, d, page, sk = 3, 8, 128, 16, 1000
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    q = torch.randn(b, sq, h, d).bfloat16().to(DEV)
    seqlens = torch.tensor([1000, 517, 33], dtype=torch.int32).to(DEV)
    paged = xfa.flash_attn_with_kvcache(q, kp.to(DEV), vp.to(DEV), cache_seqlens=seqlens,
                                        block_table=table.to(DEV), num_splits=num_splits)
    nblk = table.shape[1]
    kfull = kp[table.long().flatten()].reshape(b, nblk * page, hk, d).to(DEV)
    vfull = vp[table.long().flatten()].reshape(b, nblk * page, hk, d).to(DEV)
    dense = xfa.flash_attn_with_kvcache(q, kfull, vfull, cache_seqlens=seqlens,
                                        num_splits=num_splits)
    assert torch.equal(paged, dense)
    kpm = torch.arange(sk).view(1, -1) < seqlens.cpu().view(-1, 1)
    r, _ = orc.attention_ref(q.cpu(), kc, vc, None, kpm)
    pt, _ = orc.attention_ref(q.cpu(), kc, vc, None, kpm, upcast=False, reorder_ops=True)
    _assert_parity(paged, r, pt, mult=3.0, atol=1e-5, what="paged")


def _fp8_cache(x, scale, dt=torch.bfloat16):
    """Quantise a cache to OCP e4m3fn with a per-tensor scale; returns (fp8, dequant-as-dt)
    where dequant = dt(f32(fp8) * scale), the kernel's own conversion."""
    q8 = (x.float() / scale).clamp(-448, 448).to(torch.float8_e4m3fn)
    return q8, (q8.float() * scale).to(dt)


@pytest.mark.parametrize("num_splits", [1, 0, 3])
@pytest.mark.parametrize("sq,hk", [(1, 8), (1, 2), (4, 2), (16, 2)])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_paged_fp8_cache(xfa, num_splits, sq, hk, dtype):
    """fp8 (e4m3fn) paged cache vs the oracle over the dequantised cache dt(f32(fp8) * scale),
    within the kvcache tolerance.  (No reference counterpart: the reference has no fp8 cache —
    SURVEY §8d C5 is this build's extension; parity pinned by the dequantised-cache oracle.)
    sq * H/Hk <= 32 runs the decode kernel (scales applied in fp32 to S and O); sq = 16 runs the
    general kernel, whose staging dequantises exactly like the reference cache would, so there
    it must also equal the 16-bit path over the dequantised cache bit for bit."""
    torch.manual_seed(1)
    dt = _dtype(dtype)
    b, h, d, page, sk = 3, 8, 128, 16, 1000
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    ks, vs = 0.0123, 0.0371  # not powers of two: the dequant rounding is exercised
    kp8, kpd = _fp8_cache(kp, ks, dt)
    vp8, vpd = _fp8_cache(vp, vs, dt)
    q = torch.randn(b, sq, h, d).to(dt).to(DEV)
    seqlens = torch.tensor([1000, 517, 33], dtype=torch.int32).to(DEV)
    tab = table.to(DEV)
    out8, lse8 = xfa.flash_attn_with_kvcache(q, kp8.to(DEV), vp8.to(DEV), cache_seqlens=seqlens,
                                             block_table=tab, num_splits=num_splits,
                                             return_softmax_lse=True, k_scale=ks, v_scale=vs)
    # (the 16-bit paged cache would run the ping-pong kernel: compare with the kernel the fp8
    # cache runs, whose staging the bit-for-bit claim is about)
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    w4 = L.fmha_get_option(b"fwd_w4")
    assert L.fmha_set_option(b"fwd_w4", 0) == 0
    try:
        outd, lsed = xfa.flash_attn_with_kvcache(q, kpd.to(DEV), vpd.to(DEV), cache_seqlens=seqlens,
                                                 block_table=tab, num_splits=num_splits,
                                                 return_softmax_lse=True)
    finally:
        L.fmha_set_option(b"fwd_w4", w4)
    if sq * h // hk > 32:
        assert torch.equal(out8, outd)
        assert torch.equal(lse8, lsed)
    else:
        assert (lse8 - lsed).abs().max().item() < 5e-3
    nblk = table.shape[1]
    kfull = kpd[table.long().flatten()].reshape(b, nblk * page, hk, d)[:, :sk]
    vfull = vpd[table.long().flatten()].reshape(b, nblk * page, hk, d)[:, :sk]
    kpm = torch.arange(sk).view(1, -1) < seqlens.cpu().view(-1, 1)
    r, _ = orc.attention_ref(q.cpu(), kfull, vfull, None, kpm)
    pt, _ = orc.attention_ref(q.cpu(), kfull, vfull, None, kpm, upcast=False, reorder_ops=True)
    _assert_parity(out8, r, pt, mult=3.0, atol=1e-5, what="paged fp8")
    _assert_parity(outd, r, pt, mult=3.0, atol=1e-5, what="paged dequantised")


def test_paged_fp8_generic_staging_bitexact(xfa):
    """With the decode kernel switched off, the general kernel's fp8 staging (dequantise while
    staging) equals the 16-bit path over the dequantised cache bit for bit."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(3)
    b, h, hk, d, page, sk = 2, 8, 2, 128, 16, 300
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    kp8, kpd = _fp8_cache(kp, 0.02)
    vp8, vpd = _fp8_cache(vp, 0.03)
    q = torch.randn(b, 1, h, d).bfloat16().to(DEV)
    seqlens = torch.tensor([300, 77], dtype=torch.int32).to(DEV)
    tab = table.to(DEV)
    assert L.fmha_set_option(b"fwd_decode", 0) == 0
    try:
        o8 = xfa.flash_attn_with_kvcache(q, kp8.to(DEV), vp8.to(DEV), cache_seqlens=seqlens,
                                         block_table=tab, k_scale=0.02, v_scale=0.03)
        od = xfa.flash_attn_with_kvcache(q, kpd.to(DEV), vpd.to(DEV), cache_seqlens=seqlens,
                                         block_table=tab)
    finally:
        L.fmha_set_option(b"fwd_decode", 1)
    assert torch.equal(o8, od)


@pytest.mark.parametrize("sq,h,hk,d", [(1, 32, 8, 128), (1, 8, 1, 64), (2, 16, 2, 128),
                                       (1, 6, 6, 64), (3, 12, 1, 128)])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_decode_kernel_dense(xfa, sq, h, hk, d, causal, dtype):
    """Decode shapes (sq * H/Hk <= 32) through mha_fwd (dense K/V) and through the paged cache,
    against the oracle; the decode and general kernels agree to rounding."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(5)
    b, sk = 3, 777
    q = torch.randn(b, sq, h, d, dtype=dtype)
    k = torch.randn(b, sk, hk, d, dtype=dtype)
    v = torch.randn(b, sk, hk, d, dtype=dtype)
    out = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=causal)
    r, _ = orc.attention_ref(q, k, v, causal=causal)
    pt, _ = orc.attention_ref(q, k, v, causal=causal, upcast=False, reorder_ops=True)
    _assert_parity(out, r, pt, what="decode dense")
    assert L.fmha_set_option(b"fwd_decode", 0) == 0
    try:
        ref_gen = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=causal)
    finally:
        L.fmha_set_option(b"fwd_decode", 1)
    assert (out.float() - ref_gen.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("sq,h,hk", [(1, 32, 8), (3, 12, 1), (2, 64, 2)])
def test_decode_folded_combine_bitexact(xfa, sq, h, hk):
    """dec_fold=1 (the last split of each (b, kv head) merges the partials in the decode
    launch) gives the same output and LSE as the separate per-wave combine kernel
    (comb_row=0: the same serial order over splits), bit for bit, twice in a row (the split
    counters reset themselves); the default one-workgroup-per-row combine (comb_row=1) sums
    the splits in groups, equal up to fp32 reassociation."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(8)
    b, d, sk = 3, 128, 1500
    q = torch.randn(b, sq, h, d, dtype=torch.bfloat16).to(DEV)
    k = torch.randn(b, sk, hk, d, dtype=torch.bfloat16).to(DEV)
    v = torch.randn(b, sk, hk, d, dtype=torch.bfloat16).to(DEV)
    row = xfa.flash_attn_func(q, k, v, causal=True, return_attn_probs=True)
    # (shapes past the decode kernel's 32 rows run the split kernel + combine either way)
    assert L.fmha_set_option(b"comb_row", 0) == 0
    try:
        base = xfa.flash_attn_func(q, k, v, causal=True, return_attn_probs=True)
        assert L.fmha_set_option(b"dec_fold", 1) == 0
        for _ in range(2):
            f = xfa.flash_attn_func(q, k, v, causal=True, return_attn_probs=True)
            assert torch.equal(f[0], base[0]) and torch.equal(f[1], base[1])
    finally:
        L.fmha_set_option(b"dec_fold", 0)
        L.fmha_set_option(b"comb_row", 1)
    _assert_ulps(row[0].float(), base[0].float(), 2, torch.bfloat16, 2.0 ** -20)
    _assert_ulps(row[1], base[1], 2, torch.float32)


@pytest.mark.parametrize("window", [(64, 0), (100, 7), (-1, 5)])
def test_decode_kernel_window_alibi_softcap(xfa, window):
    torch.manual_seed(6)
    b, sq, h, hk, d, sk = 2, 4, 16, 4, 128, 500
    q = torch.randn(b, sq, h, d, dtype=torch.bfloat16)
    k = torch.randn(b, sk, hk, d, dtype=torch.bfloat16)
    v = torch.randn(b, sk, hk, d, dtype=torch.bfloat16)
    slopes = torch.rand(b, h, dtype=torch.float32) * 0.3
    bias = orc.alibi_bias(slopes, sq, sk, causal=False)
    win = oracle_window(window, sk)
    out = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), window_size=window,
                              alibi_slopes=slopes.to(DEV), softcap=15.0)
    r, _ = orc.attention_ref(q, k, v, attn_bias=bias, window_size=win, softcap=15.0)
    pt, _ = orc.attention_ref(q, k, v, attn_bias=bias, window_size=win, softcap=15.0,
                              upcast=False, reorder_ops=True)
    _assert_parity(out, r, pt, mult=5.0, what=f"decode window {window}")


def test_paged_fp8_capi(xfa):
    """fmha_page_kvcache_fwd_ex(kv_dtype=1) through the C ABI == the pybind fp8 op, bitwise;
    an unknown kv_dtype is rejected."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(2)
    b, h, hk, d, page, sk = 2, 8, 2, 128, 16, 256
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    kp8, _ = _fp8_cache(kp, 0.02)
    vp8, _ = _fp8_cache(vp, 0.03)
    q = torch.randn(b, 1, h, d).bfloat16().to(DEV)
    seqlens = torch.tensor([256, 100], dtype=torch.int32).to(DEV)
    tab, k8, v8 = table.to(DEV), kp8.to(DEV), vp8.to(DEV)
    ref = xfa.flash_attn_with_kvcache(q, k8, v8, cache_seqlens=seqlens, block_table=tab,
                                      k_scale=0.02, v_scale=0.03, num_splits=1)
    out = torch.empty_like(q)
    lse = torch.empty(b, h, 1, device=DEV, dtype=torch.float32)
    args = [q.data_ptr(), k8.data_ptr(), v8.data_ptr(), out.data_ptr(), lse.data_ptr(),
            tab.data_ptr(), tab.stride(0), seqlens.data_ptr(), 1, sk, b, h, hk, d, page,
            d ** -0.5, -1, -1, 0.0, None, 0, 1]
    st = capi.stream_handle()
    L.fmha_page_kvcache_fwd_ex(*args, 1, 0.02, 0.03, None, 0, st)
    torch.cuda.synchronize()
    assert L.fmha_last_status() == 0, L.fmha_last_error()
    assert torch.equal(out, ref)
    L.fmha_page_kvcache_fwd_ex(*args, 7, 1.0, 1.0, None, 0, st)
    assert L.fmha_last_status() != 0
    assert b"kv_dtype" in L.fmha_last_error()


@pytest.mark.parametrize("paged", [True, False])
@pytest.mark.parametrize("rotary_fraction", [0.0, 0.5, 1.0])
@pytest.mark.parametrize("rotary_interleaved", [False, True])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("mha_type", ["mha", "gqa"])
@pytest.mark.parametrize("seqlen_q,seqlen_k", [(1, 128), (3, 339), (64, 256)])
def test_kvcache_append(xfa, paged, rotary_fraction, rotary_interleaved, causal, mha_type,
                        seqlen_q, seqlen_k):
    """Append new K/V (+ rotary) into the cache, then attend: the recipe of the reference's
    test_flash_attn_kvcache with new_kv=True (test.py:1355-1594), whose rotary branch is
    commented out there — rotary parity is pinned by oracle.apply_rotary only."""
    if rotary_fraction == 0.0 and rotary_interleaved:
        pytest.skip("interleaving is meaningless without rotary")
    torch.manual_seed(0)
    dtype = torch.bfloat16
    b, h, d = 2, 6, 128
    hk = h if mha_type == "mha" else 3
    rotary_dim = int(rotary_fraction * d) // 16 * 16
    seqlen_new = seqlen_q
    q = torch.randn(b, seqlen_q, h, d, dtype=dtype)
    k = torch.randn(b, seqlen_new, hk, d, dtype=dtype)
    v = torch.randn(b, seqlen_new, hk, d, dtype=dtype)
    page = 16
    if paged:
        kc, vc, table, kp, vp, nblk = orc.block_kvcache(seqlen_k, page, b, hk, d, dtype=dtype)
    else:
        kc = torch.randn(b, seqlen_k, hk, d, dtype=dtype)
        vc = torch.randn(b, seqlen_k, hk, d, dtype=dtype)
    hi = seqlen_k - (seqlen_q if causal and rotary_dim > 0 else seqlen_new) + 1
    cache_seqlens = torch.randint(0, hi, (b,), dtype=torch.int32)
    arange = torch.arange(seqlen_k).view(1, -1)
    cs = cache_seqlens.view(-1, 1)
    kpm = arange < cs + seqlen_new
    if rotary_dim > 0:
        angle = torch.rand(seqlen_k if not paged else nblk * page, rotary_dim // 2) * 2 * math.pi
        cos, sin = torch.cos(angle).to(dtype), torch.sin(angle).to(dtype)
        if causal:
            q_ro = orc.apply_rotary(q, cos, sin, cache_seqlens, rotary_interleaved)
        else:
            q_ro = orc.apply_rotary(q.reshape(b, 1, seqlen_q * h, d), cos, sin, cache_seqlens,
                                    rotary_interleaved).reshape(b, seqlen_q, h, d)
        k_ro = orc.apply_rotary(k, cos, sin, cache_seqlens, rotary_interleaved)
    else:
        cos = sin = None
        q_ro, k_ro = q, k
    upd = (cs <= arange) & (arange < cs + seqlen_new)
    k_ref, v_ref = kc.clone(), vc.clone()
    k_ref[upd] = k_ro.reshape(-1, hk, d)
    v_ref[upd] = v.reshape(-1, hk, d)
    kd = (kp if paged else kc).clone().to(DEV)
    vd = (vp if paged else vc).clone().to(DEV)
    out = xfa.flash_attn_with_kvcache(
        q.to(DEV), kd, vd, k.to(DEV), v.to(DEV),
        rotary_cos=None if cos is None else cos.to(DEV),
        rotary_sin=None if sin is None else sin.to(DEV),
        cache_seqlens=cache_seqlens.to(DEV), block_table=table.to(DEV) if paged else None,
        causal=causal, rotary_interleaved=rotary_interleaved)
    torch.cuda.synchronize()
    if paged:
        nb = table.shape[1]
        ksel = kd.cpu()[table.long().flatten()].reshape(b, nb * page, hk, d)[:, :seqlen_k]
        vsel = vd.cpu()[table.long().flatten()].reshape(b, nb * page, hk, d)[:, :seqlen_k]
    else:
        ksel, vsel = kd.cpu(), vd.cpu()
    assert torch.allclose(ksel.float(), k_ref.float(), rtol=1e-3, atol=1e-3)
    assert torch.equal(vsel, v_ref)
    r, _ = orc.attention_ref(q_ro, k_ref, v_ref, None, kpm, causal=causal)
    pt, _ = orc.attention_ref(q_ro, k_ref, v_ref, None, kpm, causal=causal, upcast=False,
                              reorder_ops=True)
    _assert_parity(out, r, pt, mult=3.0, atol=1e-5, what="kvcache append")


@pytest.mark.parametrize("new_kv", [False, True])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("alibi", [False, True])
@pytest.mark.parametrize("seqlen_q,seqlen_k,hk,d", [(1, 128, 2, 128), (1, 339, 6, 64),
                                                    (3, 339, 3, 128), (64, 256, 1, 128)])
def test_kvcache_leftpad(xfa, new_kv, causal, alibi, seqlen_q, seqlen_k, hk, d):
    """cache_leftpad on a dense cache, the recipe of the reference's test_flash_attn_kvcache with
    has_leftpad=True (test.py:1427-1436, parametrised off there, test.py:1333): batch b's keys
    are cache rows [leftpad[b], cache_seqlens[b] (+ new)), positions counted from leftpad[b]
    (oracle key_leftpad, test.py:258-261,286-289).  seqlen_q = 1 runs the decode kernel."""
    torch.manual_seed(1)
    dtype = torch.bfloat16
    b, h = 2, 6
    q = torch.randn(b, seqlen_q, h, d, dtype=dtype)
    kc = torch.randn(b, seqlen_k, hk, d, dtype=dtype)
    vc = torch.randn(b, seqlen_k, hk, d, dtype=dtype)
    seqlen_new = seqlen_q if new_kv else 0
    cache_seqlens = torch.randint(0 if new_kv else 1, seqlen_k - seqlen_new + 1, (b,),
                                  dtype=torch.int32)
    leftpad = torch.cat([torch.randint(0, int(c), (1,), dtype=torch.int32) if c > 0
                         else torch.zeros(1, dtype=torch.int32) for c in cache_seqlens])
    arange = torch.arange(seqlen_k).view(1, -1)
    cs = cache_seqlens.view(-1, 1)
    kpm = (arange < cs + seqlen_new) & (arange >= leftpad.view(-1, 1))
    k_ref, v_ref = kc.clone(), vc.clone()
    k = v = None
    if new_kv:
        k = torch.randn(b, seqlen_new, hk, d, dtype=dtype)
        v = torch.randn(b, seqlen_new, hk, d, dtype=dtype)
        upd = (cs <= arange) & (arange < cs + seqlen_new)
        k_ref[upd] = k.reshape(-1, hk, d)
        v_ref[upd] = v.reshape(-1, hk, d)
    slopes = torch.rand(b, h, dtype=torch.float32) * 0.3 if alibi else None
    bias = orc.alibi_bias(slopes, seqlen_q, seqlen_k, None, kpm, causal=causal,
                          key_leftpad=leftpad) if alibi else None
    kd, vd = kc.clone().to(DEV), vc.clone().to(DEV)
    out = xfa.flash_attn_with_kvcache(
        q.to(DEV), kd, vd, None if k is None else k.to(DEV), None if v is None else v.to(DEV),
        cache_seqlens=cache_seqlens.to(DEV), cache_leftpad=leftpad.to(DEV), causal=causal,
        alibi_slopes=None if slopes is None else slopes.to(DEV))
    torch.cuda.synchronize()
    r, _ = orc.attention_ref(q, k_ref, v_ref, None, kpm, bias, causal=causal, key_leftpad=leftpad)
    pt, _ = orc.attention_ref(q, k_ref, v_ref, None, kpm, bias, causal=causal, upcast=False,
                              reorder_ops=True, key_leftpad=leftpad)
    _assert_parity(out, r, pt, mult=3.0, atol=1e-5, what="kvcache leftpad")


def test_kvcache_leftpad_paged_rejected(xfa):
    """As flash-attn: no paged KV with leftpad (export.cpp:1628, commented out there)."""
    q = torch.randn(1, 1, 4, 64, dtype=torch.float16, device=DEV)
    kc = torch.randn(4, 16, 4, 64, dtype=torch.float16, device=DEV)
    table = torch.arange(4, dtype=torch.int32, device=DEV).view(1, 4)
    lens = torch.tensor([40], dtype=torch.int32, device=DEV)
    lp = torch.tensor([3], dtype=torch.int32, device=DEV)
    with pytest.raises(NotImplementedError):
        xfa.flash_attn_with_kvcache(q, kc, kc, cache_seqlens=lens, block_table=table,
                                    cache_leftpad=lp)
    with pytest.raises(RuntimeError, match="leftpad"):
        paged_attn = xfa.interface.paged_attn
        paged_attn.fwd_kvcache(q, kc, kc, None, None, lens, None, None, None, table, None, None,
                               0.125, False, -1, -1, 0.0, False, 0, lp)


def test_kvcache_cache_batch_idx(xfa):
    """Dense cache indexed through cache_batch_idx (batch b reads cache row idx[b])."""
    torch.manual_seed(4)
    b, bc, h, d, sk = 2, 5, 4, 64, 200
    q = torch.randn(b, 1, h, d, dtype=torch.float16)
    kc = torch.randn(bc, sk, h, d, dtype=torch.float16)
    vc = torch.randn(bc, sk, h, d, dtype=torch.float16)
    idx = torch.tensor([3, 1], dtype=torch.int32)
    lens = torch.tensor([200, 57], dtype=torch.int32)
    out = xfa.flash_attn_with_kvcache(q.to(DEV), kc.to(DEV), vc.to(DEV), cache_seqlens=lens.to(DEV),
                                      cache_batch_idx=idx.to(DEV))
    ks, vs = kc[idx.long()], vc[idx.long()]
    kpm = torch.arange(sk).view(1, -1) < lens.view(-1, 1)
    r, _ = orc.attention_ref(q, ks, vs, None, kpm)
    pt, _ = orc.attention_ref(q, ks, vs, None, kpm, upcast=False, reorder_ops=True)
    _assert_parity(out, r, pt, mult=3.0, atol=1e-5, what="cache_batch_idx")


# ------------------------------------------------------------ persistent forward: item order ---
@pytest.mark.parametrize("cfg", [
    dict(b=2, h=32, hk=8, s=2048, d=128, causal=True),
    dict(b=2, h=32, hk=32, s=2048, d=64, causal=True),
    dict(b=2, h=16, hk=16, s=3000, d=128, causal=False),
    dict(b=1, h=32, hk=4, s=4093, d=96, causal=True),
    dict(b=2, h=16, hk=16, s=2048, d=128, causal=False, window=(300, 0)),
    dict(b=2, h=16, hk=16, s=2048, d=128, causal=False, window=(-1, 100)),
])
def test_fwd_persistent_order_bitexact(xfa, cfg):
    """Persistent grid (items > resident workgroups): the XCD-grouped item order changes neither
    bits of O nor of the LSE (an item's arithmetic does not depend on where it runs), and the
    result stays within the reference rule of the oracle."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(11)
    b, h, hk, s, d = cfg["b"], cfg["h"], cfg["hk"], cfg["s"], cfg["d"]
    q = torch.randn(b, s, h, d, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(b, s, hk, d, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(b, s, hk, d, device=DEV, dtype=torch.bfloat16)
    window = cfg.get("window", (-1, -1))
    outs = []
    try:
        # boustrophedon, XCD-grouped pairs, and the dynamic item queue (twice: the queue's
        # device counter must have reset itself after the first launch)
        for order, dyn, xq in ((0, 1, 1), (1, 1, 1), (1, 2, 1), (1, 2, 1), (1, 2, 0)):
            assert L.fmha_set_option(b"fwd_order", order) == 0
            assert L.fmha_set_option(b"fwd_dyn", dyn) == 0
            assert L.fmha_set_option(b"fwd_xcdq", xq) == 0
            o, lse = xfa.flash_attn_func(q, k, v, causal=cfg["causal"], window_size=window,
                                         return_attn_probs=True)[:2]
            outs.append((o.clone(), lse.clone()))
    finally:
        L.fmha_set_option(b"fwd_order", 1)
        L.fmha_set_option(b"fwd_dyn", 1)
        L.fmha_set_option(b"fwd_xcdq", 1)
    for o, lse in outs[1:]:
        assert torch.equal(o, outs[0][0])
        assert torch.equal(lse, outs[0][1])
    if True:                                  # oracle on the first 4 query heads of batch 0
        qs, ks, vs = q[:1, :, :4], k[:1, :, :max(1, 4 * hk // h)], v[:1, :, :max(1, 4 * hk // h)]
        r, _ = orc.attention_ref(qs.float(), ks.float(), vs.float(), causal=cfg["causal"],
                                 window_size=window)
        pt, _ = orc.attention_ref(qs, ks, vs, causal=cfg["causal"], window_size=window,
                                  upcast=False, reorder_ops=True)
        _assert_parity(outs[-1][0][:1, :, :4].float().cpu(), r.cpu(), pt.float().cpu(),
                       what=str(cfg))


@pytest.mark.parametrize("causal", [True, False])
def test_fwd_varlen_dynamic_queue_bitexact(xfa, causal):
    """Varlen runs the dynamic item queue by default (fwd_dyn=1): same bits as the static
    persistent order, launch after launch (the counter resets itself), and the oracle's rule."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(12)
    h, d = 16, 128
    lens = [1900, 37, 1024, 1500, 2000, 256, 999, 1777]        # 1024 row-block items > 256 CUs
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    q, k, v = (torch.randn(sum(lens), h, d, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    outs = []
    try:
        for dyn, xq in ((0, 1), (1, 1), (1, 1), (1, 0), (1, 0)):
            assert L.fmha_set_option(b"fwd_dyn", dyn) == 0
            assert L.fmha_set_option(b"fwd_xcdq", xq) == 0
            o = xfa.flash_attn_varlen_func(q, k, v, cu, cu, max(lens), max(lens), causal=causal)
            outs.append(o.clone())
    finally:
        L.fmha_set_option(b"fwd_dyn", 1)
        L.fmha_set_option(b"fwd_xcdq", 1)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    for i in (1, 4):                                      # two sequences against the oracle
        s0, s1 = int(cu[i]), int(cu[i + 1])
        qs, ks, vs = (x[s0:s1, :4][None].cpu() for x in (q, k, v))
        r, _ = orc.attention_ref(qs.float(), ks.float(), vs.float(), causal=causal)
        pt, _ = orc.attention_ref(qs, ks, vs, causal=causal, upcast=False, reorder_ops=True)
        _assert_parity(outs[-1][s0:s1, :4][None].float().cpu(), r, pt.float(), what=f"seq{i}")


# ------------------------------------------------------------------- head dims 129..256 ---
# The reference dispatches head-dim buckets up to 256 (static_switch.h:90-117); D in
# (128, 256] runs the 4-wave, 512-register build of the forward kernel.
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [136, 160, 192, 256])
@pytest.mark.parametrize("sq,sk,h,hk", [(1, 147, 4, 4), (113, 203, 4, 2), (300, 300, 6, 3),
                                        (1023, 1024, 2, 2)])
def test_fwd_large_head_dims(xfa, dtype, causal, d, sq, sk, h, hk):
    q, k, v, out_ref, out_pt = _rand_case(1, h, hk, sq, sk, d, dtype, causal, seed=d)
    out, lse, _ = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), causal=causal,
                                      return_attn_probs=True)
    assert out.shape == (1, sq, h, d)
    _assert_parity(out, out_ref, out_pt, what=f"{sq}x{sk} h{h}/{hk} d{d} c{causal}")
    lse_ref = orc.attention_lse_ref(q, k, causal=causal)
    fin = torch.isfinite(lse_ref)
    assert torch.equal(torch.isinf(lse.cpu()), ~fin)
    assert (lse.cpu()[fin] - lse_ref[fin]).abs().max().item() < LSE_ATOL


@pytest.mark.parametrize("window", [(17, 3), (-1, 40)])
def test_fwd_d256_windows_alibi_softcap(xfa, window):
    torch.manual_seed(3)
    b, h, hk, sq, sk, d = 2, 4, 2, 211, 333, 256
    q = torch.randn(b, sq, h, d).bfloat16()
    k = torch.randn(b, sk, hk, d).bfloat16()
    v = torch.randn(b, sk, hk, d).bfloat16()
    slopes = torch.rand(b, h) * 0.3
    w = oracle_window(window, sk)
    bias = orc.alibi_bias(slopes, sq, sk, causal=False)
    r, _ = orc.attention_ref(q, k, v, attn_bias=bias, window_size=w, softcap=30.0)
    pt, _ = orc.attention_ref(q, k, v, attn_bias=bias, window_size=w, softcap=30.0,
                              upcast=False, reorder_ops=True)
    out = xfa.flash_attn_func(q.to(DEV), k.to(DEV), v.to(DEV), window_size=window,
                              softcap=30.0, alibi_slopes=slopes.to(DEV))
    _assert_parity(out, r, pt, what=f"d256 window {window} alibi softcap")


@pytest.mark.parametrize("splits", [2, 5])
def test_fwd_d256_split_kv(xfa, splits):
    torch.manual_seed(1)
    q = torch.randn(2, 64, 4, 256, dtype=torch.bfloat16, device=DEV)
    k = torch.randn(2, 1500, 2, 256, dtype=torch.bfloat16, device=DEV)
    v = torch.randn(2, 1500, 2, 256, dtype=torch.bfloat16, device=DEV)
    one = xfa.flash_attn_with_kvcache(q, k, v, causal=True, num_splits=1)
    many = xfa.flash_attn_with_kvcache(q, k, v, causal=True, num_splits=splits)
    assert (one.float() - many.float()).abs().max().item() < 2e-2
    r, _ = orc.attention_ref(q.cpu(), k.cpu(), v.cpu(), causal=True)
    pt, _ = orc.attention_ref(q.cpu(), k.cpu(), v.cpu(), causal=True, upcast=False, reorder_ops=True)
    _assert_parity(many, r, pt, mult=3.0, atol=1e-5, what=f"d256 splits {splits}")


def test_varlen_d192(xfa):
    torch.manual_seed(2)
    h, hk, d = 4, 1, 192
    lq, lk = [1, 257, 64, 700], [90, 257, 1, 700]
    cu_q = torch.tensor([0] + list(torch.tensor(lq).cumsum(0)), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(lk).cumsum(0)), dtype=torch.int32)
    q = torch.randn(sum(lq), h, d).half()
    k = torch.randn(sum(lk), hk, d).half()
    v = torch.randn(sum(lk), hk, d).half()
    for causal in (False, True):
        out = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cu_q.to(DEV),
                                         cu_k.to(DEV), max(lq), max(lk), causal=causal).cpu()
        for i in range(len(lq)):
            qs = q[cu_q[i]:cu_q[i + 1]][None]
            ks, vs = k[cu_k[i]:cu_k[i + 1]][None], v[cu_k[i]:cu_k[i + 1]][None]
            r, _ = orc.attention_ref(qs, ks, vs, causal=causal)
            pt, _ = orc.attention_ref(qs, ks, vs, causal=causal, upcast=False, reorder_ops=True)
            _assert_parity(out[cu_q[i]:cu_q[i + 1]][None], r, pt, what=f"d192 seq {i} c{causal}")


@pytest.mark.parametrize("sq", [1, 5])
def test_paged_d256_bitexact(xfa, sq):
    """Paged decode at D = 256 (general kernel, split-KV) == dense gather, bit for bit."""
    torch.manual_seed(4)
    b, h, hk, d, page, sk = 3, 8, 2, 256, 16, 700
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    q = torch.randn(b, sq, h, d).bfloat16().to(DEV)
    seqlens = torch.tensor([700, 301, 17], dtype=torch.int32).to(DEV)
    paged = xfa.flash_attn_with_kvcache(q, kp.to(DEV), vp.to(DEV), cache_seqlens=seqlens,
                                        block_table=table.to(DEV))
    nblk = table.shape[1]
    kfull = kp[table.long().flatten()].reshape(b, nblk * page, hk, d).to(DEV)
    vfull = vp[table.long().flatten()].reshape(b, nblk * page, hk, d).to(DEV)
    dense = xfa.flash_attn_with_kvcache(q, kfull, vfull, cache_seqlens=seqlens)
    assert torch.equal(paged, dense)
    kpm = torch.arange(sk).view(1, -1) < seqlens.cpu().view(-1, 1)
    r, _ = orc.attention_ref(q.cpu(), kc, vc, None, kpm)
    pt, _ = orc.attention_ref(q.cpu(), kc, vc, None, kpm, upcast=False, reorder_ops=True)
    _assert_parity(paged, r, pt, mult=3.0, atol=1e-5, what="paged d256")


def test_d256_backward_over_256_rejected(xfa):
    q = torch.randn(1, 64, 2, 264, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="at most 256"):
        xfa.flash_attn_func(q, q, q, causal=True)


def test_varlen_reference_signature_capi(xfa):
    """fmha_varlen_fwd with the reference's own signature (csrc/paged_attn.h:33-53,
    paged_attn.cpp:385-440; causality from the windows only, is_causal ignored) through ctypes:
    bitwise equal to the pybind varlen op and within the oracle rule per sequence."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(21)
    h, hk, d = 6, 2, 128
    lq, lk = [1, 300, 77, 513], [147, 300, 600, 513]
    cu_q = torch.tensor([0] + list(torch.tensor(lq).cumsum(0)), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(lk).cumsum(0)), dtype=torch.int32)
    q = torch.randn(sum(lq), h, d).bfloat16()
    k = torch.randn(sum(lk), hk, d).bfloat16()
    v = torch.randn(sum(lk), hk, d).bfloat16()
    qd, kd, vd, cqd, ckd = (x.to(DEV) for x in (q, k, v, cu_q, cu_k))
    for wl, wr, causal in ((-1, 0, True), (-1, -1, False), (64, 8, False)):
        ref_out = xfa.flash_attn_varlen_func(qd, kd, vd, cqd, ckd, max(lq), max(lk),
                                             causal=causal, window_size=(wl, wr) if not causal else (-1, -1))
        o = torch.empty_like(qd)
        L.fmha_varlen_fwd(qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), o.data_ptr(),
                          cqd.data_ptr(), ckd.data_ptr(), max(lq), max(lk), len(lq), h, hk, d,
                          capi.stream_handle(), d ** -0.5, not causal, False, wl, wr)
        capi.check()
        torch.cuda.synchronize()
        assert torch.equal(o, ref_out), (wl, wr)
        for i in range(len(lq)):
            a, b = int(cu_q[i]), int(cu_q[i + 1])
            c_, e = int(cu_k[i]), int(cu_k[i + 1])
            w = oracle_window((wl, wr), e - c_)
            r, _ = orc.attention_ref(q[a:b][None], k[c_:e][None], v[c_:e][None], window_size=w)
            pt, _ = orc.attention_ref(q[a:b][None], k[c_:e][None], v[c_:e][None], window_size=w,
                                      upcast=False, reorder_ops=True)
            _assert_parity(o[a:b][None], r, pt, what=f"ref-sig varlen seq{i} w({wl},{wr})")


def test_page_kvcache_reference_signature_capi(xfa):
    """fmha_page_kvcache_fwd with the reference's own signature (csrc/paged_attn.h:55-84,
    paged_attn.cpp:442-568): block-table row stride = max_cache_seq_k / page, seqlen_k = the
    longest cache, cache_seqlens non-cumulative; k/v/rotary/cache_batch_idx ignored as the
    reference does.  With seqlen_k = the table's capacity (what the pybind op passes,
    export.cpp:1703) it is bitwise equal to the pybind kvcache op (the split heuristic sees the
    same length); within the kvcache rule."""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    torch.manual_seed(22)
    b, h, hk, d, page, sk = 3, 8, 2, 128, 16, 1000
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    max_cache = table.shape[1] * page
    for sq in (1, 4):
        q = torch.randn(b, sq, h, d).bfloat16()
        seqlens = torch.tensor([1000, 517, 33], dtype=torch.int32)
        qd, kpd, vpd, td, sd = (x.to(DEV) for x in (q, kp, vp, table, seqlens))
        for causal, splits in ((False, 0), (True, 3)):
            ref_out = xfa.flash_attn_with_kvcache(qd, kpd, vpd, cache_seqlens=sd, block_table=td,
                                                  causal=causal, num_splits=splits)
            o = torch.empty_like(qd)
            L.fmha_page_kvcache_fwd(qd.data_ptr(), kpd.data_ptr(), vpd.data_ptr(), None, None,
                                    o.data_ptr(), td.data_ptr(), sd.data_ptr(), max_cache, sq,
                                    max_cache, b, h, hk, d, page, capi.stream_handle(), d ** -0.5,
                                    -1, 0 if (causal and sq > 1) else -1, splits, None, None,
                                    None, causal, False, False)
            capi.check()
            torch.cuda.synchronize()
            assert torch.equal(o, ref_out), (sq, causal, splits)
            kpm = torch.arange(sk).view(1, -1) < seqlens.view(-1, 1)
            r, _ = orc.attention_ref(q, kc, vc, None, kpm, causal=causal and sq > 1)
            pt, _ = orc.attention_ref(q, kc, vc, None, kpm, causal=causal and sq > 1, upcast=False,
                                      reorder_ops=True)
            _assert_parity(o, r, pt, mult=3.0, atol=1e-5, what=f"ref-sig kvcache sq{sq} c{causal}")
    # a page size that does not divide the table stride argument is the caller's contract;
    # a non-positive page size is rejected loudly
    L.fmha_page_kvcache_fwd(qd.data_ptr(), kpd.data_ptr(), vpd.data_ptr(), None, None,
                            o.data_ptr(), td.data_ptr(), sd.data_ptr(), max_cache, 4, sk, b, h,
                            hk, d, 0, capi.stream_handle(), d ** -0.5, -1, -1, 0, None, None,
                            None, False, False, False)
    assert L.fmha_last_status() != 0

"""GPU parity of the fp8 (e4m3fn) Q/K/V forward (fp8 MFMA for both GEMMs; an extension the
reference lacks, so parity is pinned by the oracle's restatement only: see
oracle.attention_fp8_pt).

Rule (the reference's shape, test.py:975): max|out - out_ref| <= 3 x max|out_pt - out_ref|,
where out_ref = the fp32 oracle over the dequantised inputs and out_pt = the same with P rounded
to e4m3 before PV (the fp8 analogue of the reference's rounding of P to the input dtype) and
its output rounded to the output dtype.  The
LSE, which never sees the e4m3 rounding of P, is held to 1e-3.
"""
import pytest
import torch

from oracle import attention_ref as orc
from tests.fp8_model import attention_fp8_kernel_model

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


def _case(b, h, hk, sq, sk, seed, amp=1.0):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(b, sq, h, 128, generator=g) * amp
    k = torch.randn(b, sk, hk, 128, generator=g) * amp
    v = torch.randn(b, sk, hk, 128, generator=g)
    return [orc.quantize_fp8(x) for x in (q, k, v)]


def _check(xfa, b, h, hk, sq, sk, causal=False, window=(-1, -1), seed=0, out_dtype=torch.bfloat16,
           amp=1.0, report=None):
    (q8, qs), (k8, ks), (v8, vs) = _case(b, h, hk, sq, sk, seed, amp)
    out, lse = xfa.flash_attn_fp8_func(q8.to(DEV), k8.to(DEV), v8.to(DEV), qs, ks, vs,
                                       causal=causal, window_size=window, out_dtype=out_dtype,
                                       return_lse=True)
    torch.cuda.synchronize()
    if window[0] < 0 or window[0] >= sk:
        _assert_fp8_w4()
    qd, kd, vd = q8.float() * qs, k8.float() * ks, v8.float() * vs
    w = (window[0], sk) if window[0] >= 0 and window[1] < 0 else window
    ref, _ = orc.attention_ref(qd, kd, vd, causal=causal, window_size=w)
    # the estimate also rounds its output to out_dtype, as the reference's pt path returns the
    # input dtype
    pt = orc.attention_fp8_pt(q8, k8, v8, qs, ks, vs, causal=causal, window_size=w).to(out_dtype)
    ok, err, bound = orc.parity_ok(out.cpu().float(), ref, pt, 3.0, 1e-3)
    if report:
        row = {"case": f"fp8 fwd b{b} h{h}/{hk} {sq}x{sk} c{causal} w{window}", "err": err,
               "bound": bound, "ok": bool(ok)}
        if _w4_ran():
            # the error of the kernel's own arithmetic (tests/fp8_model.py: P against the tile-0
            # reference max, not the row max): the cause of the cases close to their bound
            mdl = attention_fp8_kernel_model(q8, k8, v8, qs, ks, vs, causal=causal,
                                             window_size=w).to(out_dtype)
            row["model_err"] = (mdl.float() - ref).abs().max().item()
        report(row)
    assert ok, f"max|out-ref|={err:.3g} > {bound:.3g}"
    lref = orc.attention_lse_ref(qd, kd, causal=causal, window_size=w)
    fin = torch.isfinite(lref)
    assert torch.equal(torch.isinf(lse.cpu()), ~fin)
    assert (lse.cpu()[fin] - lref[fin]).abs().max().item() < 1e-3
    return out


def _w4_ran():
    from xf_flash_attention_cutlass_amd import capi
    return capi.lib().fmha_last_kernel().decode().startswith("fmha_fwd8w_kernel")


def _assert_fp8_w4():
    """launches without a left window run the generated fp8 kernel fp8_w4 selects (2 the ping-pong
    kernel, 1 the 4-wave kernel; 0, under XFA_TEST_OPTIONS=fp8_w4=0, the 8-wave compiler-scheduled
    one)"""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    kern = L.fmha_last_kernel().decode()
    want = {0: "fmha_fwd_fp8_kernel", 1: "fmha_fwd8w_kernel", 2: "fmha_fwd8pp_kernel"}
    assert kern.startswith(want[L.fmha_get_option(b"fp8_w4")]), kern


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("b,h,hk,sq,sk", [(2, 4, 4, 300, 300), (1, 8, 2, 1024, 1024),
                                          (2, 4, 1, 113, 203), (1, 2, 2, 1, 777),
                                          (1, 4, 2, 600, 250)])
def test_fp8_fwd(xfa, causal, b, h, hk, sq, sk, parity_report):
    _check(xfa, b, h, hk, sq, sk, causal=causal, report=parity_report)


@pytest.mark.parametrize("window", [(64, 0), (100, 17), (-1, 40), (0, 0)])
def test_fp8_fwd_windows(xfa, window, parity_report):
    _check(xfa, 2, 4, 2, 333, 411, window=window, seed=3, report=parity_report)


def test_fp8_fwd_fp16_out_and_large_scores(xfa, parity_report):
    # |scores| up to ~60: the deferred rescale keeps P <= 2^8 < 448 (e4m3 max)
    _check(xfa, 1, 4, 4, 512, 512, causal=True, seed=5, out_dtype=torch.float16, amp=2.5,
           report=parity_report)


def test_fp8_fwd_routing_and_capi(xfa):
    """flash_attn_func with float8 inputs routes to the fp8 kernel; the C ABI gives the same
    bytes; invalid head sizes fail loudly."""
    from xf_flash_attention_cutlass_amd import capi
    (q8, qs), (k8, ks), (v8, vs) = _case(2, 4, 2, 200, 260, 7)
    q8, k8, v8 = q8.to(DEV), k8.to(DEV), v8.to(DEV)
    a = xfa.flash_attn_func(q8, k8, v8, causal=True, q_descale=qs, k_descale=ks, v_descale=vs)
    out = torch.empty(2, 200, 4, 128, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(2, 4, 200, device=DEV)
    L = capi.lib()
    L.fmha_fwd_fp8(q8.data_ptr(), k8.data_ptr(), v8.data_ptr(), out.data_ptr(), lse.data_ptr(),
                   qs, ks, vs, 200, 260, 2, 4, 2, 128, 128 ** -0.5, -1, 0, False,
                   capi.stream_handle())
    capi.check()
    torch.cuda.synchronize()
    assert torch.equal(a, out)
    L.fmha_fwd_fp8(q8.data_ptr(), k8.data_ptr(), v8.data_ptr(), out.data_ptr(), None,
                   qs, ks, vs, 200, 260, 2, 4, 2, 64, 0.125, -1, 0, False, capi.stream_handle())
    assert L.fmha_last_status() != 0 and b"128" in L.fmha_last_error()


def test_fp8_fwd_c2_shape(xfa, parity_report):
    """The C2 shape in fp8 (B4 H32 S4096 causal): sampled heads against the oracle, every head
    bit-identical between the persistent and the one-workgroup-per-item schedules."""
    from xf_flash_attention_cutlass_amd import capi
    B, S, H = 4, 4096, 32
    g = torch.Generator(device=DEV).manual_seed(9)
    x = [torch.randn(B, S, H, 128, device=DEV, generator=g) for _ in range(3)]
    q8s = [orc.quantize_fp8(t) for t in x]
    (q8, qs), (k8, ks), (v8, vs) = q8s
    out = xfa.flash_attn_fp8_func(q8, k8, v8, qs, ks, vs, causal=True)
    _assert_fp8_w4()
    for bb, hh in ((0, 0), (3, 31)):
        sl = [t[bb:bb + 1, :, hh:hh + 1].cpu() for t in (q8, k8, v8)]
        ref, _ = orc.attention_ref(*(t.float() * s for t, s in zip(sl, (qs, ks, vs))), causal=True)
        pt = orc.attention_fp8_pt(*sl, qs, ks, vs, causal=True).bfloat16()
        ok, err, bound = orc.parity_ok(out[bb:bb + 1, :, hh:hh + 1].cpu().float(), ref, pt, 3.0, 1e-3)
        parity_report({"case": f"fp8 C2 b{bb} h{hh}", "err": err, "bound": bound, "ok": bool(ok)})
        assert ok, f"b{bb} h{hh}: {err:.3g} > {bound:.3g}"
    L = capi.lib()
    assert L.fmha_set_option(b"fwd_persistent", 0) == 0
    try:
        out_np = xfa.flash_attn_fp8_func(q8, k8, v8, qs, ks, vs, causal=True)
    finally:
        L.fmha_set_option(b"fwd_persistent", 1)
    assert torch.equal(out, out_np)
    # the per-XCD dynamic item queues (fwd_dyn = 2), twice (the counters reset themselves)
    dyn = L.fmha_get_option(b"fwd_dyn")
    assert L.fmha_set_option(b"fwd_dyn", 2) == 0
    try:
        for _ in range(2):
            out_dyn = xfa.flash_attn_fp8_func(q8, k8, v8, qs, ks, vs, causal=True)
            assert "persistent=3" in L.fmha_last_kernel().decode() or not L.fmha_get_option(b"fp8_w4")
            assert torch.equal(out, out_dyn)
    finally:
        L.fmha_set_option(b"fwd_dyn", dyn)

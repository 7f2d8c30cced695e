"""GPU: the generated D = 128 forward kernels the knobs select.

fwd_w4 = 1 (4-wave, csrc/fmha_fwd4_kernel.h), 2 (8-wave ping-pong, csrc/fmha_fwdpp_kernel.h)
and 3 (the ping-pong on v_mfma_f32_16x16x32, tools/gen_fwdpp16.py; 4 = auto, the default, picks
3 or 2 by mask); fp8_w4 = 1 (4-wave fp8, the default) and 2 (ping-pong fp8,
csrc/fmha_fwd8pp_kernel.h).  The kernels no default path runs (fwd_w4 = 1, fp8_w4 = 2) live only
in the variants build (lib/variants/libpaged-attention.so, build.py: XFA_VARIANTS=1), which these
tests load next to the product library through the same C ABI.  Each setting runs the same
cases: the kernel id is asserted (fmha_last_kernel), the output is held to the oracle by the
reference's rule (test.py:975), and the two kernels of a pair must agree bit for bit - they
compute every row with the same tile order, reference max and operation order, only the
row-to-wave split and the schedule differ.  The 16x16x32 ping-pong sums each MFMA's products in
another order, so it is held to the oracle (O) and to the 32x32x16 kernel's LSE within 1e-4.
"""
import pytest
import torch

from oracle import attention_ref as orc
from tests import test_fwd4_redo_gpu as r4

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


_VAR = {}


def _variants():
    """the variants build, loaded once (ctypes; its soname differs from the product's)"""
    if "lib" not in _VAR:
        from xf_flash_attention_cutlass_amd import capi
        _VAR["lib"] = capi.load(capi.VARIANTS_PATH)
    return _VAR["lib"]


def _run(lib, fn):
    from xf_flash_attention_cutlass_amd import capi
    fn()
    if lib.fmha_last_status() != 0:
        raise RuntimeError(lib.fmha_last_error().decode())
    torch.cuda.synchronize()
    return lib.fmha_last_kernel().decode()


def _fwd_lib(lib, w4, q, k, v, causal, window=(-1, -1)):
    """fmha_fwd of `lib` with fwd_w4 = w4, one split: (O, LSE); asserts the kernel that ran"""
    from xf_flash_attention_cutlass_amd import capi
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    q, k, v = (x.to(DEV).contiguous() for x in (q, k, v))
    o = torch.empty_like(q)
    lse = torch.empty(b, h, sq, device=DEV, dtype=torch.float32)
    wl, wr = (-1, 0) if causal else window
    old = lib.fmha_get_option(b"fwd_w4")
    assert lib.fmha_set_option(b"fwd_w4", w4) == 0, lib.fmha_last_error()
    try:
        kern = _run(lib, lambda: lib.fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, sq, sk,
                                              b, h, hk, d, 0.0, capi.stream_handle(), None, d ** -0.5, None,
                                              lse.data_ptr(), wl, wr, 0.0, False, q.dtype == torch.float16, 1))
    finally:
        lib.fmha_set_option(b"fwd_w4", old)
    assert kern.startswith(r4.expected_kernel(w4, wr) + " "), kern
    return o.cpu(), lse.cpu()


def test_product_refuses_variant_kernels():
    """the product library has no fwd_w4 = 1 / fp8_w4 = 2 kernels and says so"""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    assert L.fmha_set_option(b"fwd_w4", 1) != 0 and b"variants" in L.fmha_last_error()
    assert L.fmha_set_option(b"fp8_w4", 2) != 0 and b"variants" in L.fmha_last_error()
    V = _variants()
    assert b"variants" in V.fmha_version()


BF16_CASES = [
    # b, h, hk, sq, sk, causal, window
    (2, 4, 4, 700, 700, True, (-1, -1)),
    (1, 8, 2, 513, 1025, False, (-1, -1)),
    (2, 4, 4, 300, 900, True, (-1, -1)),
    (1, 4, 4, 1024, 1024, False, (-1, 200)),    # right window only (a left one: 8-wave kernel)
]


def _pair(q, k, v, causal, window):
    """4-wave (variants) vs ping-pong (variants and product): oracle + bit identity"""
    from xf_flash_attention_cutlass_amd import capi
    o1 = _fwd_lib(_variants(), 1, q, k, v, causal, window)
    o2 = _fwd_lib(_variants(), 2, q, k, v, causal, window)
    o2p = _fwd_lib(capi.lib(), 2, q, k, v, causal, window)
    ref, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window)
    pt, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window, upcast=False, reorder_ops=True)
    ok, err, bound = orc.parity_ok(o2[0].float(), ref, pt, 2.0, 1e-5)
    assert ok, f"max|out-ref| = {err:.3g} > {bound:.3g}"
    for x, y in ((o1, o2), (o2, o2p)):
        assert torch.equal(x[0], y[0]) and torch.equal(x[1], y[1])


@pytest.mark.parametrize("b,h,hk,sq,sk,causal,window", BF16_CASES)
def test_fwd_w4_kernels_agree(b, h, hk, sq, sk, causal, window):
    g = torch.Generator().manual_seed(sq + sk)
    q = torch.randn(b, sq, h, 128, generator=g).bfloat16()
    k = torch.randn(b, sk, hk, 128, generator=g).bfloat16()
    v = torch.randn(b, sk, hk, 128, generator=g).bfloat16()
    _pair(q, k, v, causal, window)


FP8_CASES = [
    # b, h, hk, sq, sk, causal
    (2, 4, 2, 700, 700, True),
    (1, 8, 8, 513, 1025, False),
    (2, 4, 4, 300, 900, True),
]


def _fp8_lib(lib, w4, b, h, hk, sq, sk, causal, seed):
    """fmha_fwd_fp8 of `lib` with fp8_w4 = w4 (bf16 out), checked against the fp8 oracle
    estimate (tests/test_fp8_gpu.py's rule); returns O"""
    from xf_flash_attention_cutlass_amd import capi
    from tests import test_fp8_gpu as f8
    (q8, qs), (k8, ks), (v8, vs) = f8._case(b, h, hk, sq, sk, seed)
    qd8, kd8, vd8 = (x.to(DEV) for x in (q8, k8, v8))
    o = torch.empty(b, sq, h, 128, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(b, h, sq, device=DEV, dtype=torch.float32)
    old = lib.fmha_get_option(b"fp8_w4")
    assert lib.fmha_set_option(b"fp8_w4", w4) == 0, lib.fmha_last_error()
    try:
        kern = _run(lib, lambda: lib.fmha_fwd_fp8(qd8.data_ptr(), kd8.data_ptr(), vd8.data_ptr(), o.data_ptr(),
                                                  lse.data_ptr(), qs, ks, vs, sq, sk, b, h, hk, 128,
                                                  128 ** -0.5, -1, 0 if causal else -1, False,
                                                  capi.stream_handle()))
    finally:
        lib.fmha_set_option(b"fp8_w4", old)
    assert kern.startswith({1: "fmha_fwd8w_kernel ", 2: "fmha_fwd8pp_kernel "}[w4]), kern
    qd, kd, vd = q8.float() * qs, k8.float() * ks, v8.float() * vs
    ref, _ = orc.attention_ref(qd, kd, vd, causal=causal)
    pt = orc.attention_fp8_pt(q8, k8, v8, qs, ks, vs, causal=causal).to(torch.bfloat16)
    ok, err, bound = orc.parity_ok(o.cpu().float(), ref, pt, 3.0, 1e-3)
    assert ok, f"fp8 max|out-ref|={err:.3g} > {bound:.3g}"
    return o.cpu()


@pytest.mark.parametrize("b,h,hk,sq,sk,causal", FP8_CASES)
def test_fp8_w4_kernels_agree(b, h, hk, sq, sk, causal):
    from xf_flash_attention_cutlass_amd import capi
    o1 = _fp8_lib(_variants(), 1, b, h, hk, sq, sk, causal, sq)
    o2 = _fp8_lib(_variants(), 2, b, h, hk, sq, sk, causal, sq)
    o1p = _fp8_lib(capi.lib(), 1, b, h, hk, sq, sk, causal, sq)
    assert torch.equal(o1, o2) and torch.equal(o1, o1p)


def _sweep(n, seed):
    """seeded random shapes around the edges the kernels special-case: lengths below one key
    tile, at and just past 64 / 256 multiples, sq > sk (rows with no key under causal), GQA
    groups 1-8, right windows, fp16"""
    g = torch.Generator().manual_seed(seed)
    lens = [1, 17, 63, 64, 65, 255, 256, 257, 383, 512, 777]
    out = []
    for _ in range(n):
        pick = lambda xs: xs[int(torch.randint(len(xs), (1,), generator=g))]  # noqa: E731
        hk = pick([1, 2, 4])
        grp = pick([1, 2, 4, 8]) if hk < 4 else pick([1, 2])
        mode = pick(["causal", "none", "right"])
        window = (-1, pick([0, 5, 100])) if mode == "right" else (-1, -1)
        sq = pick(lens)
        if sq * grp <= 32:        # a whole GQA group in one 32-row tile: the decode kernel's
            continue
        out.append((pick([1, 2]), hk * grp, hk, sq, pick(lens), mode == "causal", window,
                    pick([torch.bfloat16, torch.float16])))
    return out


@pytest.mark.parametrize("b,h,hk,sq,sk,causal,window,dt", _sweep(20, 5))
def test_fwd_w4_kernels_sweep(b, h, hk, sq, sk, causal, window, dt):
    g = torch.Generator().manual_seed(b * 1000 + sq * 7 + sk)
    q = torch.randn(b, sq, h, 128, generator=g).to(dt)
    k = torch.randn(b, sk, hk, 128, generator=g).to(dt)
    v = torch.randn(b, sk, hk, 128, generator=g).to(dt)
    _pair(q, k, v, causal, window)


def _sweep8(n, seed):
    g = torch.Generator().manual_seed(seed)
    lens = [17, 64, 65, 255, 256, 257, 511, 777]
    out = []
    for _ in range(n):
        pick = lambda xs: xs[int(torch.randint(len(xs), (1,), generator=g))]  # noqa: E731
        hk = pick([1, 2, 4])
        out.append((pick([1, 2]), hk * pick([1, 2, 4]), hk, pick(lens), pick(lens), bool(pick([0, 1]))))
    return out


@pytest.mark.parametrize("b,h,hk,sq,sk,causal", _sweep8(10, 11))
def test_fp8_w4_kernels_sweep(b, h, hk, sq, sk, causal):
    o1 = _fp8_lib(_variants(), 1, b, h, hk, sq, sk, causal, sk)
    o2 = _fp8_lib(_variants(), 2, b, h, hk, sq, sk, causal, sk)
    assert torch.equal(o1, o2)


def _check16(q, k, v, causal, window):
    """fwd_w4 = 3 against the oracle (O, reference rule) and the fwd_w4 = 2 LSE; returns (O, LSE)"""
    from xf_flash_attention_cutlass_amd import capi
    outs = {w4: _fwd_lib(capi.lib(), w4, q, k, v, causal, window) for w4 in (2, 3, 4)}
    assert torch.equal(outs[4][0], outs[3 if window[1] < 0 and not causal else 2][0])
    ref, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window)
    pt, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window, upcast=False, reorder_ops=True)
    ok, err, bound = orc.parity_ok(outs[3][0].float(), ref, pt, 2.0, 1e-5)
    assert ok, f"16x16: max|out-ref| = {err:.3g} > {bound:.3g}"
    l2, l3 = outs[2][1], outs[3][1]
    assert torch.equal(torch.isinf(l2), torch.isinf(l3))
    fin = torch.isfinite(l2)
    assert (l2[fin] - l3[fin]).abs().max().item() <= 1e-4
    return outs[3]


@pytest.mark.parametrize("b,h,hk,sq,sk,causal,window", BF16_CASES)
def test_fwd_w4_16x16_cases(b, h, hk, sq, sk, causal, window):
    g = torch.Generator().manual_seed(sq + sk)
    q = torch.randn(b, sq, h, 128, generator=g).bfloat16()
    k = torch.randn(b, sk, hk, 128, generator=g).bfloat16()
    v = torch.randn(b, sk, hk, 128, generator=g).bfloat16()
    _check16(q, k, v, causal, window)


@pytest.mark.parametrize("b,h,hk,sq,sk,causal,window,dt", _sweep(20, 5) + _sweep(12, 23))
def test_fwd_w4_16x16_sweep(b, h, hk, sq, sk, causal, window, dt):
    g = torch.Generator().manual_seed(b * 1000 + sq * 7 + sk)
    q = torch.randn(b, sq, h, 128, generator=g).to(dt)
    k = torch.randn(b, sk, hk, 128, generator=g).to(dt)
    v = torch.randn(b, sk, hk, 128, generator=g).to(dt)
    _check16(q, k, v, causal, window)


@pytest.mark.parametrize("opts", [(("fwd_persistent", 1), ("fwd_order", 0)),
                                  (("fwd_persistent", 1), ("fwd_order", 1)),
                                  (("fwd_persistent", 1), ("fwd_dyn", 2))])
def test_fwd_w4_multi_item_schedules(opts):
    """more items than CUs (4 x 16 heads x 8 row blocks = 512 items), so each persistent
    workgroup reuses its LDS ring across items: the 4-wave and ping-pong kernels stay bit
    identical under every schedule, the 16x16x32 one meets the oracle on samples"""
    V = _variants()
    g = torch.Generator().manual_seed(99)
    b, h, s = 4, 16, 2048
    q = torch.randn(b, s, h, 128, generator=g).bfloat16()
    k = torch.randn(b, s, h, 128, generator=g).bfloat16()
    v = torch.randn(b, s, h, 128, generator=g).bfloat16()
    olds = {n: V.fmha_get_option(n.encode()) for n, _ in opts}
    try:
        for n, val in opts:
            assert V.fmha_set_option(n.encode(), val) == 0
        o1 = _fwd_lib(V, 1, q, k, v, True)
        o2 = _fwd_lib(V, 2, q, k, v, True)
        o3 = _fwd_lib(V, 3, q, k, v, False)
    finally:
        for n, val in olds.items():
            V.fmha_set_option(n.encode(), val)
    assert torch.equal(o1[0], o2[0]) and torch.equal(o1[1], o2[1])
    for bb, hh in ((0, 0), (3, 15)):
        qs, ks, vs = (x[bb:bb + 1, :, hh:hh + 1] for x in (q, k, v))
        ref, _ = orc.attention_ref(qs, ks, vs, causal=False)
        pt, _ = orc.attention_ref(qs, ks, vs, causal=False, upcast=False, reorder_ops=True)
        ok, err, bound = orc.parity_ok(o3[0][bb:bb + 1, :, hh:hh + 1].float(), ref, pt, 2.0, 1e-5)
        assert ok, f"16x16 multi-item ({bb}, {hh}): {err:.3g} > {bound:.3g}"


@pytest.mark.parametrize("causal", [True, False])
def test_fwdpp_varlen_seqused_k(xfa, causal):
    """varlen with seqused_k (each sequence reads only the first seqused_k[b] of its keys, the
    non-paged per-sequence key limit of flash-attn's varlen path): that route into the
    ping-pong kernels, against the oracle per sequence"""
    from xf_flash_attention_cutlass_amd import capi
    pa = xfa.paged_attn
    g = torch.Generator().manual_seed(123)
    h, hk = 8, 4
    lq, lk, used = [300, 129, 500], [1000, 300, 777], [1000, 17, 600]
    cq = torch.tensor([0] + list(torch.tensor(lq).cumsum(0)), dtype=torch.int32)
    ck = torch.tensor([0] + list(torch.tensor(lk).cumsum(0)), dtype=torch.int32)
    q = torch.randn(int(cq[-1]), h, 128, generator=g).bfloat16()
    k = torch.randn(int(ck[-1]), hk, 128, generator=g).bfloat16()
    v = torch.randn(int(ck[-1]), hk, 128, generator=g).bfloat16()
    r = pa.varlen_fwd(q.to(DEV), k.to(DEV), v.to(DEV), None, cq.to(DEV), ck.to(DEV),
                      torch.tensor(used, dtype=torch.int32, device=DEV), None, None, max(lq), max(lk),
                      0.0, 128 ** -0.5, False, causal, -1, -1, 0.0, False, None)
    torch.cuda.synchronize()
    out = r[0].cpu()
    kern = capi.lib().fmha_last_kernel().decode()
    assert kern.startswith(r4.expected_kernel(capi.lib().fmha_get_option(b"fwd_w4"),
                                              0 if causal else -1) + " "), kern
    for i in range(len(lq)):
        a_, b_ = int(cq[i]), int(cq[i + 1])
        c_ = int(ck[i])
        qs, ks, vs = q[a_:b_][None], k[c_:c_ + used[i]][None], v[c_:c_ + used[i]][None]
        ref, _ = orc.attention_ref(qs, ks, vs, causal=causal)
        pt, _ = orc.attention_ref(qs, ks, vs, causal=causal, upcast=False, reorder_ops=True)
        ok, err, bound = orc.parity_ok(out[a_:b_][None].float(), ref, pt, 2.0, 1e-5)
        assert ok, f"seqused_k seq {i}: {err:.3g} > {bound:.3g}"


FEAT_CASES = [
    # b, h, hk, sq, sk, causal, window, alibi, softcap
    (2, 4, 4, 700, 700, True, (-1, -1), True, 0.0),
    (1, 8, 2, 513, 1025, False, (-1, -1), True, 0.0),
    (1, 8, 2, 513, 1025, True, (-1, -1), True, 0.0),      # causal ALiBi, sq < sk: linear frame, diag > 0
    (2, 4, 4, 300, 900, True, (-1, -1), False, 30.0),
    (1, 4, 2, 1024, 1024, False, (-1, 200), True, 20.0),
    (2, 8, 8, 257, 129, True, (-1, -1), True, 15.0),     # sq > sk: rows with no key
    # left windows (sliding / local), alone and with the features
    (2, 4, 4, 1100, 1100, False, (255, 0), False, 0.0),
    (1, 8, 2, 700, 1300, False, (100, 30), False, 0.0),
    (2, 4, 2, 1300, 700, False, (64, 0), True, 0.0),      # sq > sk
    (1, 4, 4, 2048, 2048, False, (1023, 0), True, 25.0),
    (2, 4, 4, 777, 777, False, (0, 0), False, 0.0),       # the diagonal only
    (1, 4, 4, 513, 513, False, (300, -1), True, 0.0),     # left window only (right = sk)
]


@pytest.mark.parametrize("b,h,hk,sq,sk,causal,window,alibi,softcap", FEAT_CASES)
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_fwdpp_alibi_softcap(b, h, hk, sq, sk, causal, window, alibi, softcap, dt):
    """ALiBi, softcap and left windows on the 32x32x16 ping-pong kernel's score-feature pass and
    two-sided key window (the kernel id is asserted): O against the oracle (test.py:975 rule; 3x with softcap, whose tanh the oracle
    evaluates in fp32), the LSE against the fp32 log-sum-exp in the reference kernel's ALiBi form
    (mask_hip.h:162-167), and O within bf16 rounding of the compiler-scheduled 8-wave kernel"""
    from xf_flash_attention_cutlass_amd import capi
    g = torch.Generator().manual_seed(sq * 3 + sk)
    q = (torch.randn(b, sq, h, 128, generator=g) * 2).to(dt)
    k = torch.randn(b, sk, hk, 128, generator=g).to(dt)
    v = torch.randn(b, sk, hk, 128, generator=g).to(dt)
    slopes = torch.rand(b, h, generator=g) * 0.3 if alibi else None
    L = capi.lib()

    def run(w4):
        qd, kd, vd = (x.to(DEV).contiguous() for x in (q, k, v))
        o = torch.empty_like(qd)
        lse = torch.empty(b, h, sq, device=DEV, dtype=torch.float32)
        sl = slopes.to(DEV).contiguous() if alibi else None
        wl, wr = (-1, 0) if causal else window
        old = L.fmha_get_option(b"fwd_w4")
        assert L.fmha_set_option(b"fwd_w4", w4) == 0
        try:
            kern = _run(L, lambda: L.fmha_fwd(qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), o.data_ptr(),
                                              sl.data_ptr() if alibi else None, sq, sk, b, h, hk, 128, 0.0,
                                              capi.stream_handle(), None, 128 ** -0.5, None, lse.data_ptr(),
                                              wl, wr, softcap, False, dt == torch.float16, 1))
        finally:
            L.fmha_set_option(b"fwd_w4", old)
        return o.cpu(), lse.cpu(), kern

    o, lse, kern = run(4)
    assert kern.startswith("fmha_fwdpp_kernel "), kern
    o8, _, kern8 = run(0)
    assert kern8.startswith("fmha_fwd_kernel"), kern8
    bias_o = orc.alibi_bias(slopes, sq, sk, causal=causal) if alibi else None
    w = (-1, 0) if causal else (window[0], sk) if window[0] >= 0 and window[1] < 0 else window
    ref, _ = orc.attention_ref(q, k, v, attn_bias=bias_o, causal=causal, window_size=w, softcap=softcap)
    pt, _ = orc.attention_ref(q, k, v, attn_bias=bias_o, causal=causal, window_size=w, softcap=softcap,
                              upcast=False, reorder_ops=True)
    ok, err, bound = orc.parity_ok(o.float(), ref, pt, 3.0 if softcap else 2.0, 1e-5)
    assert ok, f"O: max|out-ref| = {err:.3g} > {bound:.3g}"
    bias_l = orc.alibi_bias_kernel(slopes, sq, sk, causal=causal) if alibi else None
    lref = orc.attention_lse_ref(q, k, attn_bias=bias_l, causal=causal, window_size=w, softcap=softcap)
    fin = torch.isfinite(lref)
    assert torch.equal(torch.isinf(lse), ~fin)
    assert (lse[fin] - lref[fin]).abs().max().item() < 1e-3
    assert (o.float() - o8.float()).abs().max().item() <= 4 * (pt.float() - ref).abs().max().item() + 1e-2


@pytest.mark.parametrize("window,alibi", [((127, 0), True), ((300, 40), False), ((0, 0), False)])
def test_fwdpp_varlen_left_window(window, alibi):
    """Left windows on ragged varlen sequences through the ping-pong kernel (each sequence's item
    key range starts at its first row's window: the per-sequence T0 shift), with ALiBi; O per
    sequence against the oracle (test.py:975 rule), LSE against the fp32 log-sum-exp"""
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    g = torch.Generator().manual_seed(11 + window[0])
    lens = [1, 65, 300, 700, 129, 513]
    h, hk = 4, 2
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    tot = int(cu[-1])
    q = (torch.randn(tot, h, 128, generator=g) * 2).bfloat16()
    k, v = (torch.randn(tot, hk, 128, generator=g).bfloat16() for _ in range(2))
    slopes = torch.rand(len(lens), h, generator=g) * 0.3 if alibi else None
    out, lse, _ = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cu.to(DEV), cu.to(DEV),
                                             max(lens), max(lens), window_size=window,
                                             alibi_slopes=slopes.to(DEV) if alibi else None,
                                             return_attn_probs=True)
    torch.cuda.synchronize()
    kern = capi.lib().fmha_last_kernel().decode()
    if capi.lib().fmha_get_option(b"fwd_w4") in (2, 4):
        assert kern.startswith("fmha_fwdpp_kernel "), kern
    out, lse = out.cpu(), lse.cpu()
    for i, n in enumerate(lens):
        a, e = int(cu[i]), int(cu[i + 1])
        qs, ks, vs = q[a:e][None], k[a:e][None], v[a:e][None]
        s = slopes[i:i + 1] if alibi else None
        bias = orc.alibi_bias(s, n, n, causal=False) if alibi else None
        ref, _ = orc.attention_ref(qs, ks, vs, attn_bias=bias, window_size=window)
        pt, _ = orc.attention_ref(qs, ks, vs, attn_bias=bias, window_size=window, upcast=False,
                                  reorder_ops=True)
        ok, err, bound = orc.parity_ok(out[a:e][None].float(), ref, pt, 2.0, 1e-5)
        assert ok, f"seq {i} (len {n}): {err:.3g} > {bound:.3g}"
        lref = orc.attention_lse_ref(qs, ks, attn_bias=bias, window_size=window)[0]
        fin = torch.isfinite(lref)
        assert torch.equal(torch.isinf(lse[:, a:e]), ~fin)
        assert (lse[:, a:e][fin] - lref[fin]).abs().max().item() < 1e-3


def test_fwdpp_left_window_persistent_schedules():
    """A sliding window over more items than CUs (B4 H16 S2048, window (255, 0): 512 items):
    sampled heads against the oracle, every head bit-identical between the persistent XCD-paired
    grid, one workgroup per item and the per-XCD dynamic queues (ring slots reused across items
    with the item key range shifted per item)"""
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    B, S, H, W = 4, 2048, 16, (255, 0)
    g = torch.Generator(device=DEV).manual_seed(5)
    q, k, v = (torch.randn(B, S, H, 128, device=DEV, generator=g, dtype=torch.bfloat16) for _ in range(3))
    out = xfa.flash_attn_func(q, k, v, window_size=W)
    kern = L.fmha_last_kernel().decode()
    if L.fmha_get_option(b"fwd_w4") in (2, 4):
        assert kern.startswith("fmha_fwdpp_kernel persistent="), kern
    for b, hh in ((0, 0), (2, 7), (3, 15)):
        qs, ks, vs = (x[b:b + 1, :, hh:hh + 1].cpu() for x in (q, k, v))
        ref, _ = orc.attention_ref(qs, ks, vs, window_size=W)
        pt, _ = orc.attention_ref(qs, ks, vs, window_size=W, upcast=False, reorder_ops=True)
        ok, err, bound = orc.parity_ok(out[b:b + 1, :, hh:hh + 1].cpu().float(), ref, pt, 2.0)
        assert ok, f"b{b} h{hh}: {err:.3g} > {bound:.3g}"
    for opt, val in ((b"fwd_persistent", 0), (b"fwd_dyn", 2)):
        old = L.fmha_get_option(opt)
        assert L.fmha_set_option(opt, val) == 0
        try:
            assert torch.equal(out, xfa.flash_attn_func(q, k, v, window_size=W)), opt
        finally:
            L.fmha_set_option(opt, old)


def test_fwdpp16_noncausal_dynamic_default():
    """Dense non-causal D = 128 launches with more items than CUs run the 16x16x32 body from the
    per-XCD dynamic queues by default (fwd_dyn = 1): sampled heads against the oracle, every head
    bit-identical to the static XCD pairs (fwd_dyn = 0) and to one workgroup per item"""
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    B, S, H = 4, 2048, 16
    g = torch.Generator(device=DEV).manual_seed(8)
    q, k, v = (torch.randn(B, S, H, 128, device=DEV, generator=g, dtype=torch.bfloat16) for _ in range(3))
    out = xfa.flash_attn_func(q, k, v)
    kern = L.fmha_last_kernel().decode()
    if L.fmha_get_option(b"fwd_w4") == 4 and L.fmha_get_option(b"fwd_dyn") == 1:
        assert kern.startswith("fmha_fwdpp16_kernel persistent=3 xcdq=1"), kern
    for b, hh in ((0, 0), (3, 15)):
        qs, ks, vs = (x[b:b + 1, :, hh:hh + 1].cpu() for x in (q, k, v))
        ref, _ = orc.attention_ref(qs, ks, vs)
        pt, _ = orc.attention_ref(qs, ks, vs, upcast=False, reorder_ops=True)
        ok, err, bound = orc.parity_ok(out[b:b + 1, :, hh:hh + 1].cpu().float(), ref, pt, 2.0)
        assert ok, f"b{b} h{hh}: {err:.3g} > {bound:.3g}"
    for opt, val in ((b"fwd_dyn", 0), (b"fwd_persistent", 0)):
        old = L.fmha_get_option(opt)
        assert L.fmha_set_option(opt, val) == 0
        try:
            assert torch.equal(out, xfa.flash_attn_func(q, k, v)), opt
        finally:
            L.fmha_set_option(opt, old)


def test_fwdpp_sliding_window_dynamic_default():
    """Causal D = 128 launches with a left window that cuts the rows take the per-XCD dynamic
    queues by default (their row blocks carry equal work past the window's width, so the static
    pairs unbalance them); plain causal launches keep the static XCD pairs.  Bit-identical to the
    static pairs; sampled heads against the oracle."""
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    B, S, H, W = 4, 2048, 16, 255      # 512 row blocks: one pass (no split-KV)
    g = torch.Generator(device=DEV).manual_seed(9)
    q, k, v = (torch.randn(B, S, H, 128, device=DEV, generator=g, dtype=torch.bfloat16) for _ in range(3))
    out = xfa.flash_attn_func(q, k, v, causal=True, window_size=(W, 0))
    kern = L.fmha_last_kernel().decode()
    default = L.fmha_get_option(b"fwd_w4") == 4 and L.fmha_get_option(b"fwd_dyn") == 1
    if default:
        assert kern.startswith("fmha_fwdpp_kernel persistent=3 xcdq=1"), kern
    for b, hh in ((0, 0), (1, 15)):
        qs, ks, vs = (x[b:b + 1, :, hh:hh + 1].cpu() for x in (q, k, v))
        ref, _ = orc.attention_ref(qs, ks, vs, causal=True, window_size=(W, 0))
        pt, _ = orc.attention_ref(qs, ks, vs, causal=True, window_size=(W, 0), upcast=False, reorder_ops=True)
        ok, err, bound = orc.parity_ok(out[b:b + 1, :, hh:hh + 1].cpu().float(), ref, pt, 2.0)
        assert ok, f"b{b} h{hh}: {err:.3g} > {bound:.3g}"
    old = L.fmha_get_option(b"fwd_dyn")
    assert L.fmha_set_option(b"fwd_dyn", 0) == 0
    try:
        assert torch.equal(out, xfa.flash_attn_func(q, k, v, causal=True, window_size=(W, 0)))
        assert "persistent=2" in L.fmha_last_kernel().decode()
    finally:
        L.fmha_set_option(b"fwd_dyn", old)
    xfa.flash_attn_func(q, k, v, causal=True)
    if default:
        assert L.fmha_last_kernel().decode().startswith("fmha_fwdpp_kernel persistent=2"), "causal keeps the pairs"


PAGED_CASES = [
    # b, h, hk, sq, cache lens, page, causal, window, alibi
    (2, 4, 4, 300, [300, 300], 16, True, (-1, -1), False),
    (3, 8, 2, 129, [700, 129, 1000], 64, True, (-1, -1), False),     # chunked prefill: sq < sk
    (2, 4, 2, 513, [513, 600], 256, False, (-1, -1), False),
    (2, 4, 4, 400, [1100, 400], 32, False, (127, 0), True),          # sliding window + ALiBi
    (1, 4, 4, 777, [777], 128, True, (-1, -1), True),
    (2, 4, 4, 200, [200, 333], 48, True, (-1, -1), False),           # not a power of two: fallback
]


@pytest.mark.parametrize("b,h,hk,sq,lens,page,causal,window,alibi", PAGED_CASES)
def test_fwdpp_paged_prefill(b, h, hk, sq, lens, page, causal, window, alibi):
    """Paged-K/V prefill on the ping-pong kernel (gen_fwdpp.py PAGED: per tile each wave loads its
    page id from the block table and builds its own descriptors): O and LSE against the oracle
    per sequence, and bit-identical to the dense ping-pong kernel over the gathered cache (same
    tiles, same arithmetic).  Page sizes that are not a power of two >= 8 take the
    compiler-scheduled kernel."""
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    g = torch.Generator().manual_seed(sq + page)
    sk_max = max(lens)
    nbp = (sk_max + page - 1) // page
    q = (torch.randn(b, sq, h, 128, generator=g) * 2).bfloat16()
    kf = torch.randn(b, nbp * page, hk, 128, generator=g).bfloat16()
    vf = torch.randn(b, nbp * page, hk, 128, generator=g).bfloat16()
    perm = torch.randperm(b * nbp, generator=g)
    table = perm.view(b, nbp).int()
    kc = torch.full((b * nbp, page, hk, 128), float("nan")).bfloat16()   # rows past a sequence: NaN
    vc = torch.full((b * nbp, page, hk, 128), float("nan")).bfloat16()
    for i in range(b):
        n = lens[i]
        for pi in range((n + page - 1) // page):
            rows = min(page, n - pi * page)
            kc[table[i, pi], :rows] = kf[i, pi * page:pi * page + rows]
            vc[table[i, pi], :rows] = vf[i, pi * page:pi * page + rows]
    slopes = torch.rand(b, h, generator=g) * 0.3 if alibi else None
    seqlens = torch.tensor(lens, dtype=torch.int32)
    out, lse = xfa.flash_attn_with_kvcache(q.to(DEV), kc.to(DEV), vc.to(DEV), cache_seqlens=seqlens.to(DEV),
                                           block_table=table.to(DEV), causal=causal, window_size=window,
                                           alibi_slopes=slopes.to(DEV) if alibi else None,
                                           num_splits=1, return_softmax_lse=True)
    torch.cuda.synchronize()
    kern = L.fmha_last_kernel().decode()
    pow2 = page >= 8 and page & (page - 1) == 0
    if L.fmha_get_option(b"fwd_w4") in (2, 4):
        want = "fmha_fwdpp_paged_kernel " if pow2 else "fmha_fwd_kernel"
        assert kern.startswith(want), kern
    out, lse = out.cpu(), lse.cpu()
    w = (-1, 0) if causal else (window[0], max(lens)) if window[0] >= 0 and window[1] < 0 else window
    for i in range(b):
        n = lens[i]
        qs, ks, vs = q[i:i + 1], kf[i:i + 1, :n], vf[i:i + 1, :n]
        s = slopes[i:i + 1] if alibi else None
        bias = orc.alibi_bias(s, sq, n, causal=causal) if alibi else None
        ref, _ = orc.attention_ref(qs, ks, vs, attn_bias=bias, causal=causal, window_size=w)
        pt, _ = orc.attention_ref(qs, ks, vs, attn_bias=bias, causal=causal, window_size=w, upcast=False,
                                  reorder_ops=True)
        ok, err, bound = orc.parity_ok(out[i:i + 1].float(), ref, pt, 2.0, 1e-5)
        assert ok, f"seq {i}: {err:.3g} > {bound:.3g}"
        bl = orc.alibi_bias_kernel(s, sq, n, causal=causal) if alibi else None
        lref = orc.attention_lse_ref(qs, ks, attn_bias=bl, causal=causal, window_size=w)
        fin = torch.isfinite(lref)
        assert (lse[i:i + 1][fin] - lref[fin]).abs().max().item() < 1e-3
        if pow2 and L.fmha_get_option(b"fwd_w4") in (2, 4):
            # the dense ping-pong kernel (32x32 body) over the gathered rows: bit for bit
            # (one split, as the paged launch above: the split heuristic would pick split-KV)
            old = L.fmha_get_option(b"fwd_w4")
            assert L.fmha_set_option(b"fwd_w4", 2) == 0
            qd, kd, vd = (x.to(DEV).contiguous() for x in (qs, ks, vs))
            od = torch.empty_like(qd)
            sl = s.to(DEV).contiguous() if alibi else None
            wl, wr = (-1, 0) if causal else w
            try:
                L.fmha_fwd(qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), od.data_ptr(),
                           sl.data_ptr() if alibi else None, sq, n, 1, h, hk, 128, 0.0,
                           capi.stream_handle(), None, 128 ** -0.5, None, None, wl, wr, 0.0, False, False, 1)
                capi.check()
                torch.cuda.synchronize()
                assert L.fmha_last_kernel().decode().startswith("fmha_fwdpp_kernel ")
            finally:
                L.fmha_set_option(b"fwd_w4", old)
            assert torch.equal(od.cpu(), out[i:i + 1]), f"seq {i}: paged != dense"


@pytest.mark.parametrize("seed", range(12))
def test_fwdpp_paged_sweep(seed):
    """Seeded sweep of paged-K/V prefill shapes (page 8..512, GQA 1..8, ragged lengths, causal /
    non-causal / sliding windows, ALiBi, fp16): the paged ping-pong kernel bit for bit equal to
    the dense ping-pong kernel over the gathered cache, pages past each sequence NaN-filled"""
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    if L.fmha_get_option(b"fwd_w4") not in (2, 4):
        pytest.skip("the ping-pong kernel is not selected under these options")
    r = torch.Generator().manual_seed(1000 + seed)
    ri = lambda lo, hi: int(torch.randint(lo, hi + 1, (1,), generator=r))  # noqa: E731
    page = 2 ** ri(3, 9)
    hk = [1, 2, 4][ri(0, 2)]
    h = hk * [1, 2, 4, 8][ri(0, 3)]
    b = ri(1, 3)
    lens = [ri(1, 1500) for _ in range(b)]
    sq = ri(1, min(lens))
    sq = max(sq, 40 // (h // hk) + 1)          # keep sq * H/Hk > 32 (the prefill path, not decode)
    lens = [max(n, sq) for n in lens]
    mode = ri(0, 2)
    causal = mode == 0
    window = (-1, -1) if mode < 2 else (ri(0, 400), ri(0, 64))
    alibi = ri(0, 1) == 1
    dt = torch.float16 if ri(0, 1) else torch.bfloat16
    nbp = (max(lens) + page - 1) // page
    q = (torch.randn(b, sq, h, 128, generator=r) * 2).to(dt)
    kf = torch.randn(b, nbp * page, hk, 128, generator=r).to(dt)
    vf = torch.randn(b, nbp * page, hk, 128, generator=r).to(dt)
    table = torch.randperm(b * nbp, generator=r).view(b, nbp).int()
    kc = torch.full((b * nbp, page, hk, 128), float("nan")).to(dt)
    vc = torch.full((b * nbp, page, hk, 128), float("nan")).to(dt)
    for i, n in enumerate(lens):
        for pi in range((n + page - 1) // page):
            rows = min(page, n - pi * page)
            kc[table[i, pi], :rows] = kf[i, pi * page:pi * page + rows]
            vc[table[i, pi], :rows] = vf[i, pi * page:pi * page + rows]
    slopes = (torch.rand(b, h, generator=r) * 0.3).to(DEV) if alibi else None
    wl, wr = (-1, 0) if causal else window
    qd, kcd, vcd = q.to(DEV), kc.to(DEV), vc.to(DEV)
    o = torch.empty_like(qd)
    tab, seqlens = table.to(DEV), torch.tensor(lens, dtype=torch.int32).to(DEV)
    L.fmha_page_kvcache_fwd_ex(qd.data_ptr(), kcd.data_ptr(), vcd.data_ptr(), o.data_ptr(), None,
                               tab.data_ptr(), nbp, seqlens.data_ptr(), sq, nbp * page, b, h, hk, 128,
                               page, 128 ** -0.5, wl, wr, 0.0, slopes.data_ptr() if alibi else None, h, 1,
                               0, 1.0, 1.0, None, dt == torch.float16, capi.stream_handle())
    capi.check()
    torch.cuda.synchronize()
    kern = L.fmha_last_kernel().decode()
    assert kern.startswith("fmha_fwdpp_paged_kernel "), kern
    assert not torch.isnan(o).any()
    old = L.fmha_get_option(b"fwd_w4")
    assert L.fmha_set_option(b"fwd_w4", 2) == 0
    try:
        for i, n in enumerate(lens):
            kd, vd = kf[i:i + 1, :n].to(DEV).contiguous(), vf[i:i + 1, :n].to(DEV).contiguous()
            qi = qd[i:i + 1].contiguous()
            od = torch.empty_like(qi)
            sl = slopes[i:i + 1].contiguous() if alibi else None
            L.fmha_fwd(qi.data_ptr(), kd.data_ptr(), vd.data_ptr(), od.data_ptr(), sl.data_ptr() if alibi else None,
                       sq, n, 1, h, hk, 128, 0.0, capi.stream_handle(), None, 128 ** -0.5, None, None, wl, wr,
                       0.0, False, dt == torch.float16, 1)
            capi.check()
            torch.cuda.synchronize()
            assert L.fmha_last_kernel().decode().startswith("fmha_fwdpp_kernel "), L.fmha_last_kernel()
            assert torch.equal(od, o[i:i + 1]), (f"seq {i}: page {page} h {h}/{hk} sq {sq} lens {lens} "
                                                 f"causal {causal} window {window} alibi {alibi}")
    finally:
        L.fmha_set_option(b"fwd_w4", old)

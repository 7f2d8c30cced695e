"""GPU: the generated D = 128 forward kernels the knobs select, in the default run.

fwd_w4 = 1 (4-wave, csrc/fmha_fwd4_kernel.h) and 2 (8-wave ping-pong, csrc/fmha_fwdpp_kernel.h,
the default); fp8_w4 = 1 (4-wave fp8, the default) and 2 (ping-pong fp8,
csrc/fmha_fwd8pp_kernel.h).  Each setting runs the same cases: the kernel id is asserted
(fmha_last_kernel), the output is held to the oracle by the reference's rule (test.py:975), and
the two kernels of a pair must agree bit for bit - they compute every row with the same tile
order, reference max and operation order, only the row-to-wave split and the schedule differ.
(The whole GPU suite also runs under each non-default value: profiles/r05_knob_suite.log.)
"""
import pytest
import torch

from oracle import attention_ref as orc
from tests import test_fp8_gpu as f8
from tests import test_fwd4_redo_gpu as r4

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


BF16_CASES = [
    # b, h, hk, sq, sk, causal, window
    (2, 4, 4, 700, 700, True, (-1, -1)),
    (1, 8, 2, 513, 1025, False, (-1, -1)),
    (2, 4, 4, 300, 900, True, (-1, -1)),
    (1, 4, 4, 1024, 1024, False, (-1, 200)),    # right window only (a left one: 8-wave kernel)
]


@pytest.mark.parametrize("b,h,hk,sq,sk,causal,window", BF16_CASES)
def test_fwd_w4_kernels_agree(b, h, hk, sq, sk, causal, window):
    g = torch.Generator().manual_seed(sq + sk)
    q = torch.randn(b, sq, h, 128, generator=g).bfloat16()
    k = torch.randn(b, sk, hk, 128, generator=g).bfloat16()
    v = torch.randn(b, sk, hk, 128, generator=g).bfloat16()
    outs = {}
    for w4 in (1, 2):
        with r4._option("fwd_w4", w4):
            outs[w4] = r4._fwd(q, k, v, causal, window)     # asserts the kernel id for w4
    ref, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window)
    pt, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window, upcast=False, reorder_ops=True)
    ok, err, bound = orc.parity_ok(outs[2][0].float(), ref, pt, 2.0, 0.0)
    assert ok, f"max|out-ref| = {err:.3g} > {bound:.3g}"
    assert torch.equal(outs[1][0], outs[2][0])
    assert torch.equal(outs[1][1], outs[2][1])


FP8_CASES = [
    # b, h, hk, sq, sk, causal
    (2, 4, 2, 700, 700, True),
    (1, 8, 8, 513, 1025, False),
    (2, 4, 4, 300, 900, True),
]


@pytest.mark.parametrize("b,h,hk,sq,sk,causal", FP8_CASES)
def test_fp8_w4_kernels_agree(xfa, b, h, hk, sq, sk, causal):
    outs = {}
    for w4 in (1, 2):
        with r4._option("fp8_w4", w4):
            outs[w4] = f8._check(xfa, b, h, hk, sq, sk, causal=causal, seed=sq)  # oracle + kernel id
    assert torch.equal(outs[1], outs[2])


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
    outs = {}
    for w4 in (1, 2):
        with r4._option("fwd_w4", w4):
            outs[w4] = r4._fwd(q, k, v, causal, window)
    ref, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window)
    pt, _ = orc.attention_ref(q, k, v, causal=causal, window_size=window, upcast=False, reorder_ops=True)
    ok, err, bound = orc.parity_ok(outs[2][0].float(), ref, pt, 2.0, 1e-5)
    assert ok, f"max|out-ref| = {err:.3g} > {bound:.3g}"
    assert torch.equal(outs[1][0], outs[2][0])
    assert torch.equal(outs[1][1], outs[2][1])


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
def test_fp8_w4_kernels_sweep(xfa, b, h, hk, sq, sk, causal):
    outs = {}
    for w4 in (1, 2):
        with r4._option("fp8_w4", w4):
            outs[w4] = f8._check(xfa, b, h, hk, sq, sk, causal=causal, seed=sk)
    assert torch.equal(outs[1], outs[2])

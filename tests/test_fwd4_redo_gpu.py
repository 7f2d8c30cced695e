"""GPU parity of the 4-wave D = 128 forward's rare paths (fmha_fwd4_kernel.h, tools/gen_fwd4.py).

The 4-wave kernel keeps no row max in its key-tile loop: P = exp2(S c - m) against tile 0's max,
and a tile whose per-lane partial row sum passes 2^fwd_slack takes a hand-written rescale path
("redo": the tile's true max, O and l rescaled, the tile's softmax recomputed).  Unit-scale randn
inputs never reach it, so these cases force it:

  * fwd_slack = 0 (threshold 1): almost every tile after the first redoes, on the golden
    fixtures and on C2 / C4-shaped random cases;
  * scores growing along the keys (k row j scaled by 1 + A j / Sk) at the default slack.  With
    A = 40 the precondition asserted below holds: some row's later scores exceed tile 0's max by
    more than 128 log2 units, so exp2 against tile 0's max overflows fp32 - a finite output that
    matches the oracle proves the redo path ran (and fp16's P would overflow at 2^16 already);
  * sq > sk causal (bottom-right aligned) with whole 256-row items that see no key: the kernel's
    empty-item store path (O = 0, LSE = +inf, flash_fwd_kernel_hip.h:626-670).

Every call goes through the C ABI with num_splits = 1, the 4-wave kernel's eligibility (the split
heuristic would send small shapes to the split-KV path of the 8-wave kernel).  Pass rules are the
reference's (test.py:975, 1296): max|O - O_ref| <= 2 max|O_pt - O_ref|; LSE within 1e-3 of the
fp32 log-sum-exp (relative 1e-5 on top where scores reach ~100).
"""
import pytest
import torch

from oracle import attention_ref as orc
from tests import golden_util as gu

pytestmark = pytest.mark.gpu
DEV = "cuda"
LSE_ATOL = 1e-3


def _lib():
    from xf_flash_attention_cutlass_amd import capi
    return capi.lib()


class _option:
    """fmha_set_option for the duration of a block (process-wide knob, restored after)."""

    def __init__(self, name, value):
        self.name, self.value = name.encode(), value

    def __enter__(self):
        L = _lib()
        self.old = L.fmha_get_option(self.name)
        assert L.fmha_set_option(self.name, self.value) == 0

    def __exit__(self, *exc):
        assert _lib().fmha_set_option(self.name, self.old) == 0


def _fwd(q, k, v, causal, window=(-1, -1)):
    """fmha_fwd through ctypes, single pass (num_splits = 1): (O, LSE) on the GPU."""
    from xf_flash_attention_cutlass_amd import capi
    b, sq, h, d = q.shape
    sk, hk = k.shape[1], k.shape[2]
    q, k, v = (x.to(DEV).contiguous() for x in (q, k, v))
    o = torch.empty_like(q)
    lse = torch.empty(b, h, sq, device=DEV, dtype=torch.float32)
    wl, wr = (-1, 0) if causal else window
    _lib().fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, sq, sk, b, h,
                    hk, d, 0.0, capi.stream_handle(), None, d ** -0.5, None, lse.data_ptr(), wl,
                    wr, 0.0, False, q.dtype == torch.float16, 1)
    capi.check()
    torch.cuda.synchronize()
    assert _lib().fmha_last_num_splits() == 1
    _assert_fwd4(wr)
    return o.cpu(), lse.cpu()


def expected_kernel(w4, wr):
    """the kernel fwd_w4 = w4 selects for a call with right window wr (4, auto: the 16x16x32
    ping-pong where no row has a right window, else the 32x32x16 one)"""
    if w4 == 4:
        w4 = 3 if wr < 0 else 2
    return {0: "fmha_fwd_kernel", 1: "fmha_fwd4_kernel", 2: "fmha_fwdpp_kernel",
            3: "fmha_fwdpp16_kernel"}[w4]


def _assert_fwd4(wr=0):
    """the redo asm runs only in the generated D = 128 kernels: prove the one asked for ran
    (fwd_w4 = 1 the 4-wave kernel, 2 / 3 the ping-pong kernels, 4 auto; 0 under
    XFA_TEST_OPTIONS=fwd_w4=0, the compiler-scheduled 8-wave kernel)"""
    L = _lib()
    kern = L.fmha_last_kernel().decode()
    want = expected_kernel(L.fmha_get_option(b"fwd_w4"), wr)
    assert kern.startswith(want + " "), kern


def _check(o, lse, q, k, v, causal, what, rtol_lse=0.0, o_atol=None):
    ref, _ = orc.attention_ref(q, k, v, causal=causal)
    pt, _ = orc.attention_ref(q, k, v, causal=causal, upcast=False, reorder_ops=True)
    assert torch.isfinite(o.float()).all(), f"{what}: non-finite output"
    ok, err, bound = orc.parity_ok(o, ref, pt, 2.0)
    assert ok, f"{what}: max|out-ref|={err:.3g} > bound {bound:.3g}"
    if o_atol is not None:
        assert err <= o_atol, f"{what}: max|out-ref|={err:.3g} > {o_atol}"
    lref = orc.attention_lse_ref(q, k, causal=causal)
    fin = torch.isfinite(lref)
    assert torch.equal(torch.isinf(lse), ~fin), f"{what}: empty-row pattern differs"
    tol = LSE_ATOL + rtol_lse * lref[fin].abs()
    lerr = (lse[fin] - lref[fin]).abs()
    assert (lerr <= tol).all(), f"{what}: max|lse-ref|={lerr.max().item():.3g}"


def _randn(shape, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dtype)


def _growing(k, amp):
    """k rows scaled by 1 + amp * j / sk along the key axis (scores grow with the key)."""
    sk = k.shape[1]
    f = 1.0 + amp * torch.arange(sk, dtype=torch.float32) / sk
    return (k.float() * f[None, :, None, None]).to(k.dtype)


def _overflow_margin(q, k, causal):
    """max over rows of (max later score - tile 0's max) in log2 units: > 128 means exp2
    against tile 0's max overflows fp32, i.e. the kernel cannot be right without the redo."""
    c = q.shape[-1] ** -0.5 * 1.4426950408889634
    hk = k.shape[2]
    g = q.shape[2] // hk
    kk = k.float().repeat_interleave(g, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), kk) * c
    sq, sk = q.shape[1], k.shape[1]
    if causal:
        i = torch.arange(sq)[:, None]
        j = torch.arange(sk)[None, :]
        s = s.masked_fill(j > i + sk - sq, float("-inf"))
    m0 = s[..., :64].amax(-1)
    later = s[..., 64:].amax(-1)
    d = later - m0
    return d[torch.isfinite(d)].max().item()


# ------------------------------------------------------------ fwd_slack = 0: redo everywhere --
FWD4_GOLDEN = [n for n in gu.names("fwd") if gu.meta(n)["d"] == 128 and gu.meta(n)["sq"] > 32 and
               not gu.meta(n).get("alibi") and gu.meta(n)["softcap"] == 0 and
               tuple(gu.meta(n)["window"]) in ((-1, -1), (-1, 0))]


def test_fwd4_golden_list_nonempty():
    assert len(FWD4_GOLDEN) >= 3, FWD4_GOLDEN


@pytest.mark.parametrize("name", FWD4_GOLDEN)
def test_fwd4_slack0_golden(name):
    t, m = gu.load(name)
    with _option("fwd_slack", 0):
        o, lse = _fwd(t["q"], t["k"], t["v"], m["causal"])
    ok, err, bound = orc.parity_ok(o, t["out_ref"], t["out_pt"], 2.0)
    assert ok, f"{name}: max|out-ref|={err:.3g} > bound {bound:.3g}"
    lref = orc.attention_lse_ref(t["q"], t["k"], causal=m["causal"])
    fin = torch.isfinite(lref)
    assert (lse[fin] - lref[fin]).abs().max().item() < LSE_ATOL


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("b,h,hk,sq,sk", [(1, 4, 4, 1024, 1024), (2, 4, 1, 333, 1000),
                                          (1, 2, 2, 2048, 2048)])
def test_fwd4_slack0_random(dtype, causal, b, h, hk, sq, sk):
    q, k, v = (_randn(s, i, dtype) for i, s in enumerate(((b, sq, h, 128), (b, sk, hk, 128),
                                                            (b, sk, hk, 128))))
    with _option("fwd_slack", 0):
        o, lse = _fwd(q, k, v, causal)
    _check(o, lse, q, k, v, causal, f"slack0 {b}x{sq}x{sk} h{h}/{hk} c{causal} {dtype}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_fwd4_slack0_c2_shape(dtype):
    """The C2 shape (B4 H32 S4096 causal) with every tile through the redo path; sampled heads
    against the oracle, the rest equal to the default slack within rounding."""
    B, S, H, D = 4, 4096, 32, 128
    g = torch.Generator(device=DEV).manual_seed(21)
    q, k, v = (torch.randn(B, S, H, D, device=DEV, dtype=dtype, generator=g) for _ in range(3))
    with _option("fwd_slack", 0):
        o0, l0 = _fwd(q, k, v, True)
    o8, l8 = _fwd(q, k, v, True)
    assert (l0 - l8).abs().max().item() < 1e-4
    assert (o0.float() - o8.float()).abs().max().item() < 2e-2
    for bb, hh in ((0, 0), (3, 31)):
        qs, ks, vs = (x[bb:bb + 1, :, hh:hh + 1].cpu() for x in (q, k, v))
        _check(o0[bb:bb + 1, :, hh:hh + 1], l0[bb:bb + 1, hh:hh + 1], qs, ks, vs, True,
               f"C2 slack0 b{bb} h{hh}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [True, False])
def test_fwd4_slack0_varlen(xfa, dtype, causal):
    lens = [1, 63, 64, 65, 300, 1024, 257, 2000]
    H, HK, D = 4, 2, 128
    tot = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    q, k, v = (_randn((tot, hh, D), 30 + i, dtype) for i, hh in enumerate((H, HK, HK)))
    with _option("fwd_slack", 0):
        out, lse, _ = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cu.to(DEV),
                                                 cu.to(DEV), max(lens), max(lens), causal=causal,
                                                 return_attn_probs=True)
        _assert_fwd4(0 if causal else -1)
    torch.cuda.synchronize()
    out, lse = out.cpu(), lse.cpu()
    for i in range(len(lens)):
        a, e = int(cu[i]), int(cu[i + 1])
        _check(out[a:e][None], lse[:, a:e][None], q[a:e][None], k[a:e][None], v[a:e][None],
               causal, f"varlen slack0 seq{i} len{e - a}")


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


# ------------------------------------------------- scores growing along the keys, default slack --
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("amp", [4.0, 40.0])
def test_fwd4_growing_scores(dtype, causal, amp):
    b, h, hk, sq, sk = 2, 4, 2, 777, 1024
    q = _randn((b, sq, h, 128), 41, dtype)
    k = _growing(_randn((b, sk, hk, 128), 42, dtype), amp)
    v = _randn((b, sk, hk, 128), 43, dtype)
    margin = _overflow_margin(q, k, causal)
    assert margin > (128 if amp >= 40 else 16), f"precondition: margin {margin:.1f}"
    o, lse = _fwd(q, k, v, causal)
    _check(o, lse, q, k, v, causal, f"growing amp{amp} c{causal} {dtype}", rtol_lse=1e-5,
           o_atol=_rounding_bound(q, k, v, causal))


def _rounding_bound(q, k, v, causal):
    """A priori bound on |O - O_ref| from the kernel's two roundings: P to the input dtype before
    PV (half an ulp, u = 2^-8 bf16 / 2^-11 fp16, relative per weight: <= u max|v|) and O to the
    output dtype (<= u |O|); 5 % slack for the fp32 sums."""
    u = 2.0 ** -8 if q.dtype == torch.bfloat16 else 2.0 ** -11
    ref, _ = orc.attention_ref(q, k, v, causal=causal)
    return 1.05 * u * (v.float().abs().max().item() + ref.float().abs().max().item())


def test_fwd4_growing_scores_varlen(xfa):
    lens = [100, 1500, 64, 777]
    H, D = 4, 128
    tot = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    q = _randn((tot, H, D), 51, torch.bfloat16)
    v = _randn((tot, H, D), 53, torch.bfloat16)
    ks = []
    for i, n in enumerate(lens):
        ks.append(_growing(_randn((1, n, H, D), 60 + i, torch.bfloat16), 40.0)[0])
    k = torch.cat(ks)
    out, lse, _ = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cu.to(DEV),
                                             cu.to(DEV), max(lens), max(lens), causal=True,
                                             return_attn_probs=True)
    _assert_fwd4()
    torch.cuda.synchronize()
    out, lse = out.cpu(), lse.cpu()
    for i in range(len(lens)):
        a, e = int(cu[i]), int(cu[i + 1])
        qs, ks, vs = q[a:e][None], k[a:e][None], v[a:e][None]
        _check(out[a:e][None], lse[:, a:e][None], qs, ks, vs, True, f"varlen growing seq{i}",
               rtol_lse=1e-5, o_atol=_rounding_bound(qs, ks, vs, True))


# ------------------------------------------------------------- sq > sk causal: empty items --
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("h,hk", [(2, 2), (8, 2)])
def test_fwd4_empty_items(dtype, h, hk):
    """sq 600 > sk 100, causal bottom-right: rows 0..499 see no key.  With G = h/hk query heads
    per kv head packed into the rows, whole 256-row items are empty (ntl = 0 store path) and
    partly empty items have waves past their last key."""
    b, sq, sk = 2, 600, 100
    q, k, v = (_randn(s, 70 + i, dtype) for i, s in enumerate(((b, sq, h, 128), (b, sk, hk, 128),
                                                                 (b, sk, hk, 128))))
    o, lse = _fwd(q, k, v, True)
    assert (o[:, :500].float() == 0).all()
    assert torch.isinf(lse[:, :, :500]).all() and (lse[:, :, :500] > 0).all()
    _check(o, lse, q, k, v, True, f"empty items h{h}/{hk} {dtype}")

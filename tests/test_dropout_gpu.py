"""GPU: dropout and return_softmax (reference dropout_hip.h:14-109, philox.cuh:32-50,
flash_bwd_kernel_hip.h:430,660-663).

The kernels draw Philox keep bits over the score coordinates (fmha_common.h drop_block); the
tests check
  * the keep mask the forward returns (sign of S_dmask) equals oracle/dropout_ref.py's CPU
    Philox bit for bit, for the seed / offset of the returned rng_state;
  * the keep rate is 1 - p within the reference's tolerance (test.py:979-982: 0.01);
  * out, and dq / dk / dv through the backward (which regenerates the bits), against the
    oracle given that mask (attention_ref's dropout_mask, test.py:310-397) with the reference's
    rules (2x the low-precision error for out, 3x + 1e-5 for the gradients, test.py:975-986);
  * the returned softmax against the oracle's attention probabilities.
"""
import pytest
import torch

from oracle import attention_ref as orc
from oracle import dropout_ref as drf

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def xfa():
    import xf_flash_attention_cutlass_amd as m
    return m


def _fwd(xfa, q, k, v, p, causal, window=(-1, -1)):
    wl, wr = window
    r = xfa.paged_attn.fwd(q, k, v, None, None, p, q.shape[-1] ** -0.5, causal, wl, wr, 0.0,
                           True, None)
    out, lse, s, rng = r[0], r[5], r[6], r[7]
    return out, lse, s, [int(x) for x in rng.tolist()]


@pytest.mark.parametrize("b,h,hk,sq,sk,d,causal", [(2, 4, 2, 128, 128, 128, True),
                                                    (1, 3, 3, 113, 203, 64, False),
                                                    (2, 2, 1, 200, 77, 128, True)])
def test_dropout_mask_is_the_cpu_philox(xfa, b, h, hk, sq, sk, d, causal):
    torch.manual_seed(0)
    q = torch.randn(b, sq, h, d, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(b, sk, hk, d, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(b, sk, hk, d, device=DEV, dtype=torch.bfloat16)
    p = 0.17
    out, lse, s, (seed, offset) = _fwd(xfa, q, k, v, p, causal)
    assert s.shape == (b, h, (sq + 127) // 128 * 128, (sk + 127) // 128 * 128)
    kept = ~torch.signbit(s[:, :, :sq, :sk].float()).cpu()
    want = torch.from_numpy(drf.keep_mask(seed, offset, b, h, sq, sk, p))
    assert torch.equal(kept, want)
    # a second call advances the generator: a different mask
    _, _, s2, (seed2, offset2) = _fwd(xfa, q, k, v, p, causal)
    assert (seed2, offset2) != (seed, offset)
    assert not torch.equal(~torch.signbit(s2[:, :, :sq, :sk].float()).cpu(), kept)


def test_dropout_keep_rate(xfa):
    torch.manual_seed(1)
    b, h, s_, d, p = 2, 8, 512, 64, 0.17
    q = torch.randn(b, s_, h, d, device=DEV, dtype=torch.float16)
    out, lse, s, _ = _fwd(xfa, q, q, q, p, True)
    dropped = torch.signbit(s[:, :, :s_, :s_].float())
    valid = torch.ones(s_, s_, dtype=torch.bool, device=DEV).tril()
    frac = (dropped & valid).sum().item() / (valid.sum().item() * b * h)
    # the reference's rule (test.py:982); the byte threshold quantises 1 - p to (thr + 1) / 256
    assert abs(frac - p) <= 0.01, frac


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("b,h,hk,sq,sk,d,causal,window", [
    (2, 4, 2, 128, 128, 128, True, (-1, -1)),
    (1, 2, 2, 113, 203, 64, False, (-1, -1)),
    (1, 4, 1, 160, 160, 128, False, (40, 10)),
    (2, 2, 2, 96, 256, 256, True, (-1, -1)),
])
def test_dropout_fwd_bwd_vs_oracle(xfa, parity_report, dtype, b, h, hk, sq, sk, d, causal, window):
    torch.manual_seed(2)
    p = 0.2
    q = torch.randn(b, sq, h, d, dtype=dtype)
    k = torch.randn(b, sk, hk, d, dtype=dtype)
    v = torch.randn(b, sk, hk, d, dtype=dtype)
    dout = torch.randn(b, sq, h, d, dtype=dtype)
    qg, kg, vg = (x.to(DEV).requires_grad_(True) for x in (q, k, v))
    out, lse, s = xfa.flash_attn_func(qg, kg, vg, dropout_p=p, causal=causal, window_size=window,
                                      return_attn_probs=True)
    # dropout runs unsplit (paged_attn.cpp:180): the split heuristic must not engage
    from xf_flash_attention_cutlass_amd import capi
    assert capi.lib().fmha_last_num_splits() == 1
    mask = ~torch.signbit(s[:, :, :sq, :sk].float()).cpu()
    dq, dk, dv = torch.autograd.grad(out, (qg, kg, vg), dout.to(DEV))
    refs = []
    for upcast in (True, False):
        qq, kk, vv = (x.clone().requires_grad_(True) for x in (q, k, v))
        o, attn = orc.attention_ref(qq, kk, vv, None, None, None, p, mask, causal=causal,
                                    window_size=window, upcast=upcast, reorder_ops=not upcast)
        refs.append((o, attn, torch.autograd.grad(o, (qq, kk, vv), dout)))
    (o_ref, attn_ref, g_ref), (o_pt, attn_pt, g_pt) = refs
    err = (out.float().cpu() - o_ref.float()).abs().max().item()
    bound = 2 * (o_pt.float() - o_ref.float()).abs().max().item()
    case = f"dropout p{p} b{b} h{h}/{hk} {sq}x{sk} d{d} causal={causal} window={window} {dtype}"
    parity_report({"case": case + " out", "err": err, "bound": bound, "ok": err <= bound})
    assert err <= bound, (err, bound)
    for name, a, r, pt in zip(("dq", "dk", "dv"), (dq, dk, dv), g_ref, g_pt):
        e = (a.float().cpu() - r.float()).abs().max().item()
        bnd = 3 * (pt.float() - r.float()).abs().max().item() + 1e-5
        parity_report({"case": f"{case} {name}", "err": e, "bound": bnd, "ok": e <= bnd})
        assert e <= bnd, (name, e, bnd)
    # the returned softmax (P normalised, sign = dropped) against the oracle's probabilities
    sm = s[:, :, :sq, :sk].float().abs().cpu()
    e = (sm - attn_ref.float()).abs().max().item()
    assert e <= 2 * (attn_pt.float() - attn_ref.float()).abs().max().item() + 2 ** -8, e


def test_dropout_varlen_vs_oracle(xfa):
    torch.manual_seed(3)
    p, h, hk, d = 0.25, 4, 2, 128
    lq, lk = [77, 200, 1], [150, 200, 33]
    cq = torch.tensor([0, 77, 277, 278], dtype=torch.int32, device=DEV)
    ck = torch.tensor([0, 150, 350, 383], dtype=torch.int32, device=DEV)
    q = torch.randn(sum(lq), h, d, dtype=torch.bfloat16)
    k = torch.randn(sum(lk), hk, d, dtype=torch.bfloat16)
    v = torch.randn(sum(lk), hk, d, dtype=torch.bfloat16)
    out, lse, s = xfa.flash_attn_varlen_func(q.to(DEV), k.to(DEV), v.to(DEV), cq, ck, max(lq),
                                             max(lk), dropout_p=p, causal=True,
                                             return_attn_probs=True)
    oq = ok = 0
    for i, (a, bb) in enumerate(zip(lq, lk)):
        mask = ~torch.signbit(s[i:i + 1, :, :a, :bb].float()).cpu()
        o_ref, _ = orc.attention_ref(q[None, oq:oq + a], k[None, ok:ok + bb], v[None, ok:ok + bb],
                                     None, None, None, p, mask, causal=True)
        o_pt, _ = orc.attention_ref(q[None, oq:oq + a], k[None, ok:ok + bb], v[None, ok:ok + bb],
                                    None, None, None, p, mask, causal=True, upcast=False,
                                    reorder_ops=True)
        err = (out[oq:oq + a].float().cpu() - o_ref[0].float()).abs().max().item()
        assert err <= 2 * (o_pt.float() - o_ref.float()).abs().max().item() + 1e-6, (i, err)
        oq += a
        ok += bb


@pytest.mark.parametrize("deterministic", [False, True])
def test_dropout_varlen_fwd_bwd_vs_oracle(xfa, parity_report, deterministic):
    """Varlen forward + backward with dropout: dq / dk / dv of every sequence
    against the oracle given the kernel's mask, under the reference's 3x + 1e-5 rule."""
    torch.manual_seed(5)
    p, h, hk, d = 0.2, 4, 2, 64
    lq, lk = [64, 130, 1, 97], [150, 130, 40, 200]
    cq = torch.tensor([0] + list(torch.tensor(lq).cumsum(0)), dtype=torch.int32, device=DEV)
    ck = torch.tensor([0] + list(torch.tensor(lk).cumsum(0)), dtype=torch.int32, device=DEV)
    q = torch.randn(sum(lq), h, d, dtype=torch.bfloat16)
    k = torch.randn(sum(lk), hk, d, dtype=torch.bfloat16)
    v = torch.randn(sum(lk), hk, d, dtype=torch.bfloat16)
    dout = torch.randn(sum(lq), h, d, dtype=torch.bfloat16)
    qg, kg, vg = (x.to(DEV).requires_grad_(True) for x in (q, k, v))
    out, lse, s = xfa.flash_attn_varlen_func(qg, kg, vg, cq, ck, max(lq), max(lk), dropout_p=p,
                                             causal=True, deterministic=deterministic,
                                             return_attn_probs=True)
    dq, dk, dv = (g.float().cpu() for g in torch.autograd.grad(out, (qg, kg, vg), dout.to(DEV)))
    oq = ok = 0
    for i, (a, bb) in enumerate(zip(lq, lk)):
        mask = ~torch.signbit(s[i:i + 1, :, :a, :bb].float()).cpu()
        grads = []
        for upcast in (True, False):
            qq = q[None, oq:oq + a].clone().requires_grad_(True)
            kk = k[None, ok:ok + bb].clone().requires_grad_(True)
            vv = v[None, ok:ok + bb].clone().requires_grad_(True)
            o, _ = orc.attention_ref(qq, kk, vv, None, None, None, p, mask, causal=True,
                                     upcast=upcast, reorder_ops=not upcast)
            grads.append(torch.autograd.grad(o, (qq, kk, vv), dout[None, oq:oq + a]))
        got = (dq[oq:oq + a], dk[ok:ok + bb], dv[ok:ok + bb])
        for name, g, r, pt in zip(("dq", "dk", "dv"), got, grads[0], grads[1]):
            e = (g - r[0].float()).abs().max().item()
            bnd = 3 * (pt[0].float() - r[0].float()).abs().max().item() + 1e-5
            parity_report({"case": f"dropout varlen seq{i} {a}x{bb} det={deterministic} {name}",
                           "err": e, "bound": bnd, "ok": e <= bnd})
            assert e <= bnd, (i, name, e, bnd)
        oq += a
        ok += bb


def test_dropout_deterministic_bwd_bitwise(xfa):
    torch.manual_seed(4)
    q = torch.randn(2, 300, 4, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(2, 300, 2, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(2, 300, 2, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(2, 300, 4, 128, device=DEV, dtype=torch.bfloat16)
    gen = torch.cuda.get_rng_state()
    o1 = xfa.flash_attn_func(q, k, v, dropout_p=0.1, causal=True, deterministic=True)
    g1 = torch.autograd.grad(o1, (q, k, v), g)
    torch.cuda.set_rng_state(gen)
    o2 = xfa.flash_attn_func(q, k, v, dropout_p=0.1, causal=True, deterministic=True)
    g2 = torch.autograd.grad(o2, (q, k, v), g)
    assert torch.equal(o1, o2)
    for a, b_ in zip(g1, g2):
        assert torch.equal(a, b_)


def test_dropout_graph_capture(xfa):
    """Dropout inside a captured HIP graph (the key comes from torch's philox_cuda_state, read on
    the device): every replay draws a fresh mask, the device rng_state the forward
    writes is the key it used (the CPU Philox of that key reproduces the mask bit for bit), and
    the backward captured with that rng_state regenerates the same mask (dK / dV equal an eager
    backward given the same key; dQ differs by atomic summation order only)."""
    torch.manual_seed(4)
    b, h, hk, sq, sk, d, p = 1, 2, 2, 128, 160, 64, 0.17
    q = torch.randn(b, sq, h, d, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(b, sk, hk, d, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(b, sk, hk, d, device=DEV, dtype=torch.bfloat16)
    dout = torch.randn(b, sq, h, d, device=DEV, dtype=torch.bfloat16)
    sc = d ** -0.5

    def bwd(out, lse, rng):
        return xfa.paged_attn.bwd(dout, q, k, v, out, lse, None, None, None, None, p, sc, True,
                                  -1, -1, 0.0, False, None, rng)

    def step():
        r = xfa.paged_attn.fwd(q, k, v, None, None, p, sc, True, -1, -1, 0.0, True, None)
        out, lse, s, rng = r[0], r[5], r[6], r[7]
        g = bwd(out, lse, rng)
        return out, lse, s, rng, g[0], g[1], g[2]

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out, lse, s, rng, dq, dk, dv = step()
    keys, masks = [], []
    for _ in range(2):
        graph.replay()
        torch.cuda.synchronize()
        seed, offset = (int(x) for x in rng.tolist())
        kept = ~torch.signbit(s[:, :, :sq, :sk].float()).cpu()
        assert torch.equal(kept, torch.from_numpy(drf.keep_mask(seed, offset, b, h, sq, sk, p)))
        e = bwd(out, lse, rng.clone())
        torch.cuda.synchronize()
        assert torch.equal(e[1], dk) and torch.equal(e[2], dv)
        assert (e[0].float() - dq.float()).abs().max().item() <= 1e-2 * dq.float().abs().max().item()
        keys.append((seed, offset))
        masks.append(kept)
    assert keys[0] != keys[1]
    assert not torch.equal(masks[0], masks[1])

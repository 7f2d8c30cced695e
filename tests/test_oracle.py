"""CPU: the oracle restatement against the golden fixtures the reference's own oracle produced.

Pins oracle/attention_ref.py (restatement of test.py:247-397, 587-600, 1597-1621): the
fixtures were written by oracle/gen_golden.py from the reference functions themselves.
"""
import math

import pytest
import torch

from oracle import attention_ref as orc
from tests import golden_util as gu


@pytest.mark.parametrize("name", gu.names("fwd"))
def test_fwd_fixture_reproduced(name):
    t, m = gu.load(name)
    bias = None
    if m["alibi"]:
        bias = orc.alibi_bias(t["alibi_slopes"], m["sq"], m["sk"], causal=m["causal"])
    out_ref, _ = orc.attention_ref(t["q"], t["k"], t["v"], None, None, bias, 0.0, None,
                                   causal=m["causal"], window_size=tuple(m["window"]),
                                   softcap=m["softcap"])
    assert torch.equal(out_ref, t["out_ref"]), name
    out_pt, _ = orc.attention_ref(t["q"], t["k"], t["v"], None, None, bias, 0.0, None,
                                  causal=m["causal"], window_size=tuple(m["window"]),
                                  softcap=m["softcap"], upcast=False, reorder_ops=True)
    assert torch.equal(out_pt, t["out_pt"]), name


@pytest.mark.parametrize("name", gu.names("varlen"))
def test_varlen_fixture_reproduced(name):
    t, m = gu.load(name)
    out_ref, _ = orc.attention_ref(t["q"], t["k"], t["v"], t["query_padding_mask"],
                                   t["key_padding_mask"], None, 0.0, None, causal=m["causal"],
                                   window_size=tuple(m["window"]))
    assert torch.equal(out_ref, t["out_ref"]), name


@pytest.mark.parametrize("name", gu.names("kvcache"))
def test_kvcache_fixture_reproduced(name):
    t, m = gu.load(name)
    b, sk = m["b"], m["sk"]
    idx = t["block_table"].long().flatten()
    kc = t["k_cache_paged"][idx].reshape(b, -1, m["hk"], m["d"])[:, :sk]
    vc = t["v_cache_paged"][idx].reshape(b, -1, m["hk"], m["d"])[:, :sk]
    kpm = torch.arange(sk).view(1, -1) < t["cache_seqlens"].view(-1, 1)
    out_ref, _ = orc.attention_ref(t["q"], kc, vc, None, kpm, None, 0.0, None,
                                   causal=m["causal"], window_size=tuple(m["window"]))
    assert torch.equal(out_ref, t["out_ref"]), name


def test_c1_config_plumbing():
    """BASELINE configs[0]: mha_fwd B1 H4 S128 D64 fp32 non-causal on the CPU eager oracle."""
    t, m = gu.load("c1_fwd_fp32_b1h4s128d64")
    assert (m["b"], m["h"], m["sq"], m["d"], m["dtype"]) == (1, 4, 128, 64, "float32")
    q, k, v = t["q"], t["k"], t["v"]
    # independent fp64 restatement of the same math
    s = torch.einsum("bthd,bshd->bhts", q.double(), k.double()) / math.sqrt(64)
    o = torch.einsum("bhts,bshd->bthd", torch.softmax(s, -1), v.double())
    assert (o.float() - t["out_ref"]).abs().max().item() < 1e-5


def test_lse_ref_matches_logsumexp():
    torch.manual_seed(0)
    q, k = torch.randn(2, 17, 4, 32), torch.randn(2, 29, 2, 32)
    lse = orc.attention_lse_ref(q, k, causal=True)
    kk = orc.expand_kv(k, 4)
    s = torch.einsum("bthd,bshd->bhts", q, kk) / math.sqrt(32)
    s = s.masked_fill(orc.local_mask(17, 29, (-1, 0)), float("-inf"))
    assert torch.allclose(lse, torch.logsumexp(s, -1), atol=1e-5)


def test_lse_empty_rows_are_inf():
    q, k = torch.randn(1, 8, 1, 16), torch.randn(1, 4, 1, 16)
    lse = orc.attention_lse_ref(q, k, causal=True)   # sq > sk: top rows see no key
    assert torch.isinf(lse[0, 0, :4]).all() and (lse[0, 0, :4] > 0).all()
    assert torch.isfinite(lse[0, 0, 4:]).all()


def test_unpad_pad_roundtrip():
    torch.manual_seed(1)
    mask = orc.random_padding_mask(23, 5, mode="third")
    x = torch.randn(5, 23, 3, 8)
    xu, idx, cu, mx = orc.unpad_input(x, mask)
    assert cu.dtype == torch.int32 and cu[0] == 0 and cu[-1] == mask.sum()
    assert mx == int(mask.sum(-1).max())
    back = orc.pad_input(xu, idx, 5, 23)
    assert torch.equal(back[mask], x[mask]) and (back[~mask] == 0).all()


def test_parity_rule():
    ref = torch.zeros(4)
    ok, err, bound = orc.parity_ok(torch.full((4,), 0.01), ref, torch.full((4,), 0.006))
    assert ok and abs(bound - 0.012) < 1e-9
    ok, _, _ = orc.parity_ok(torch.full((4,), 0.02), ref, torch.full((4,), 0.006))
    assert not ok


@pytest.mark.parametrize("name", gu.names("dropout"))
def test_dropout_fixture_reproduced(name):
    """attention_ref's dropout branch (test.py:387-394) against the reference's own outputs and
    autograd gradients on a seeded keep mask (oracle/gen_golden.py case_dropout)."""
    t, m = gu.load(name)
    qq, kk, vv = (t[x].clone().requires_grad_(True) for x in ("q", "k", "v"))
    out, _ = orc.attention_ref(qq, kk, vv, None, None, None, m["p_drop"], t["dropout_mask"],
                               causal=m["causal"])
    assert torch.equal(out, t["out_ref"]), name
    grads = torch.autograd.grad(out, (qq, kk, vv), t["dout"])
    for n, g in zip(("dq", "dk", "dv"), grads):
        assert torch.equal(g, t[n + "_ref"]), f"{name}:{n}"
    assert 0.75 < t["dropout_mask"].float().mean().item() < 0.91     # keep rate ~ 1 - p

"""Generate the golden fixtures under tests/golden/ — TEST INFRASTRUCTURE ONLY.

Runs ONLY in the build container, where /root/reference exists.  It loads the
reference's own pure-PyTorch oracle functions out of /root/reference/test.py by
AST extraction (the module itself cannot be imported: it dlopens a DCU .so and
imports the absent third-party `flash_attn` at import time, test.py:15-31), runs
the reference's test recipes (seeds, shapes, windows, padding, paged caches) on
CPU and stores the reference's outputs (`out_ref` = upcast fp32 oracle, its gradients, and
for paged cases `out_pt` = the low-precision estimate) as small safetensors files.  The seeded
random inputs are not stored: their SHA-256 and the recipe are, and tests/golden_util.py
regenerates them (and recomputes the pinned low-precision twin) at load time.

It also checks that our restatement in `oracle/attention_ref.py` reproduces the
reference functions bit for bit on every case — outputs of both twins and, for the
forward cases, their autograd gradients (this is what pins the oracle).

Usage:  python oracle/gen_golden.py [--check-only]
"""
from __future__ import annotations

import argparse
import ast
import json
import math
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from oracle import attention_ref as ours  # noqa: E402

REF_TEST = "/root/reference/test.py"
GOLDEN = os.path.join(ROOT, "tests", "golden")
WANTED = ("attention_ref", "construct_local_mask", "attn_bias_from_alibi_slopes",
          "generate_random_padding_mask", "_generate_block_kvcache")


def load_reference_oracle():
    """Exec only the wanted top-level `def`s of test.py in a fresh namespace."""
    from einops import rearrange, repeat
    import torch.nn.functional as F
    with open(REF_TEST) as f:
        tree = ast.parse(f.read(), REF_TEST)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in WANTED]
    assert sorted(d.name for d in defs) == sorted(WANTED), [d.name for d in defs]
    mod = ast.Module(body=defs, type_ignores=[])
    ns = {"torch": torch, "math": math, "rearrange": rearrange, "repeat": repeat, "F": F,
          "Optional": None}
    exec(compile(mod, REF_TEST, "exec"), ns)  # noqa: S102 - reference oracle, this container only
    return ns


def _grads(out, inputs, g):
    return torch.autograd.grad(out, inputs, g)


def _save(name, tensors, meta, regen=(), derived=()):
    """Store the case; the seeded inputs in `regen` are dropped and recorded by SHA-256 (the
    tests regenerate them by the same recipe, tests/golden_util.py), `derived` tensors (the
    low-precision twin, pinned bit for bit above) are dropped and recomputed by the tests."""
    from safetensors.torch import save_file
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import digest
    os.makedirs(GOLDEN, exist_ok=True)
    tensors = {k: v.detach().contiguous().cpu() for k, v in tensors.items() if v is not None}
    meta = dict(meta, sha256={k: digest(tensors[k]) for k in regen if k in tensors})
    tensors = {k: v for k, v in tensors.items() if k not in regen and k not in derived}
    save_file(tensors, os.path.join(GOLDEN, name + ".safetensors"),
              metadata={"meta": json.dumps(meta)})


def _same(a, b, what):
    if a is None and b is None:
        return
    if not torch.equal(a, b):
        diff = (a.float() - b.float()).abs().max().item()
        raise AssertionError(f"restatement differs from reference on {what}: max|diff|={diff}")


def case_fwd(ref, name, *, b, h, hk, sq, sk, d, dtype, causal, local=False, alibi=False,
             softcap=0.0, grads=True, save=True):
    """Recipe of test_flash_attn_output (test.py:751-986), CPU, seed 0."""
    torch.random.manual_seed(0)
    window = (-1, -1) if not local else tuple(int(x) for x in torch.randint(0, sk, (2,)))
    q = torch.randn(b, sq, h, d, dtype=dtype)
    if softcap > 0:
        q = q * softcap
    k = torch.randn(b, sk, hk, d, dtype=dtype)
    v = torch.randn(b, sk, hk, d, dtype=dtype)
    slopes = bias = None
    if alibi:
        slopes = torch.rand(b, h, dtype=torch.float32) * 0.3
        bias = ref["attn_bias_from_alibi_slopes"](slopes, sq, sk, causal=causal)
        _same(ours.alibi_bias(slopes, sq, sk, causal=causal), bias, name + ":alibi")
    qg, kg, vg = (x.clone().requires_grad_(True) for x in (q, k, v))
    out_ref, _ = ref["attention_ref"](qg, kg, vg, None, None, bias, 0.0, None, causal=causal,
                                      window_size=window, softcap=softcap)
    out_pt, _ = ref["attention_ref"](qg, kg, vg, None, None, bias, 0.0, None, causal=causal,
                                     window_size=window, softcap=softcap, upcast=False,
                                     reorder_ops=True)
    mine_ref, _ = ours.attention_ref(q, k, v, None, None, bias, 0.0, None, causal=causal,
                                     window_size=window, softcap=softcap)
    mine_pt, _ = ours.attention_ref(q, k, v, None, None, bias, 0.0, None, causal=causal,
                                    window_size=window, softcap=softcap, upcast=False,
                                    reorder_ops=True)
    _same(mine_ref, out_ref.detach(), name + ":out_ref")
    _same(mine_pt, out_pt.detach(), name + ":out_pt")
    t = dict(q=q, k=k, v=v, alibi_slopes=slopes, out_ref=out_ref, out_pt=out_pt)
    if grads:
        # the reference's gradients of its fp32 oracle; the low-precision twin's gradients are
        # recomputed by the tests from the (bit-pinned) restatement, which keeps the fixtures small
        g = torch.randn_like(out_ref)
        dq, dk, dv = _grads(out_ref, (qg, kg, vg), g)
        t.update(dout=g, dq_ref=dq, dk_ref=dk, dv_ref=dv)
        # pin the restatement's gradients too (both twins) against the reference's autograd
        ref_pt = _grads(out_pt, (qg, kg, vg), g)
        for upcast, want in ((True, (dq, dk, dv)), (False, ref_pt)):
            mq, mk, mv = (x.clone().requires_grad_(True) for x in (q, k, v))
            mo, _ = ours.attention_ref(mq, mk, mv, None, None, bias, 0.0, None, causal=causal,
                                       window_size=window, softcap=softcap, upcast=upcast,
                                       reorder_ops=not upcast)
            for n, a, r in zip(("dq", "dk", "dv"), _grads(mo, (mq, mk, mv), g), want):
                _same(a, r, f"{name}:{n}_{'ref' if upcast else 'pt'}")
    meta = dict(kind="fwd", b=b, h=h, hk=hk, sq=sq, sk=sk, d=d, dtype=str(dtype).split(".")[-1],
                causal=causal, window=list(window), alibi=alibi, softcap=softcap,
                recipe="test.py:751-986 (test_flash_attn_output), CPU, manual_seed(0)")
    if save:
        _save(name, t, meta, regen=("q", "k", "v", "alibi_slopes", "dout"), derived=("out_pt",))
    return t


def case_dropout(ref, name, *, b, h, hk, sq, sk, d, dtype, causal, p_drop):
    """attention_ref's dropout branch (test.py:387-394, used by test_flash_attn_output with
    dropout_p > 0 and the kernel's S_dmask, test.py:873-935): a seeded keep mask stands in for
    the kernel's, the reference's fp32 oracle output and gradients are stored; the restatement
    is pinned against them bit for bit (both twins, outputs and gradients)."""
    torch.random.manual_seed(0)
    q = torch.randn(b, sq, h, d, dtype=dtype)
    k = torch.randn(b, sk, hk, d, dtype=dtype)
    v = torch.randn(b, sk, hk, d, dtype=dtype)
    keep = torch.rand(b, h, sq, sk) >= p_drop
    g = torch.randn(b, sq, h, d, dtype=dtype)
    outs = {}
    for up in (True, False):
        qg, kg, vg = (x.clone().requires_grad_(True) for x in (q, k, v))
        o, _ = ref["attention_ref"](qg, kg, vg, None, None, None, p_drop, keep, causal=causal,
                                    upcast=up, reorder_ops=not up)
        mq, mk, mv = (x.clone().requires_grad_(True) for x in (q, k, v))
        mo, _ = ours.attention_ref(mq, mk, mv, None, None, None, p_drop, keep, causal=causal,
                                   upcast=up, reorder_ops=not up)
        tag = "ref" if up else "pt"
        _same(mo.detach(), o.detach(), f"{name}:out_{tag}")
        rg = _grads(o, (qg, kg, vg), g)
        for n, a, r in zip(("dq", "dk", "dv"), _grads(mo, (mq, mk, mv), g), rg):
            _same(a, r, f"{name}:{n}_{tag}")
        outs[tag] = (o, *rg)
    o_ref, dq, dk, dv = outs["ref"]
    t = dict(q=q, k=k, v=v, dropout_mask=keep, dout=g, out_ref=o_ref, dq_ref=dq, dk_ref=dk,
             dv_ref=dv)
    meta = dict(kind="dropout", b=b, h=h, hk=hk, sq=sq, sk=sk, d=d,
                dtype=str(dtype).split(".")[-1], causal=causal, window=[-1, -1], p_drop=p_drop,
                softcap=0.0, alibi=False,
                recipe="test.py:310-397 attention_ref dropout branch; seeded keep mask "
                       "(torch.rand >= p), CPU, manual_seed(0)")
    _save(name, t, meta, regen=("q", "k", "v", "dropout_mask", "dout"))


def case_varlen(ref, name, *, b, h, hk, sq, sk, d, dtype, causal, local=False):
    """Recipe of test_flash_attn_varlen_output (test.py:1026-1307), CPU, seed 0."""
    torch.random.manual_seed(0)
    window = (-1, -1) if not local else tuple(int(x) for x in torch.randint(0, sk, (2,)))
    q = torch.randn(b, sq, h, d, dtype=dtype)
    k = torch.randn(b, sk, hk, d, dtype=dtype)
    v = torch.randn(b, sk, hk, d, dtype=dtype)
    qpm = ref["generate_random_padding_mask"](sq, b, "cpu", mode="random")
    kpm = ref["generate_random_padding_mask"](sk, b, "cpu", mode="random")
    out_ref, _ = ref["attention_ref"](q, k, v, qpm, kpm, None, 0.0, None, causal=causal,
                                      window_size=window)
    out_pt, _ = ref["attention_ref"](q, k, v, qpm, kpm, None, 0.0, None, causal=causal,
                                     window_size=window, upcast=False, reorder_ops=True)
    mine, _ = ours.attention_ref(q, k, v, qpm, kpm, None, 0.0, None, causal=causal,
                                 window_size=window)
    _same(mine, out_ref, name + ":out_ref")
    mine_pt, _ = ours.attention_ref(q, k, v, qpm, kpm, None, 0.0, None, causal=causal,
                                    window_size=window, upcast=False, reorder_ops=True)
    _same(mine_pt, out_pt, name + ":out_pt")
    t = dict(q=q, k=k, v=v, query_padding_mask=qpm, key_padding_mask=kpm,
             out_ref=out_ref, out_pt=out_pt)
    meta = dict(kind="varlen", b=b, h=h, hk=hk, sq=sq, sk=sk, d=d,
                dtype=str(dtype).split(".")[-1], causal=causal, window=list(window),
                recipe="test.py:1026-1307 (test_flash_attn_varlen_output), CPU, manual_seed(0)")
    _save(name, t, meta, regen=("q", "k", "v"), derived=("out_pt",))


def case_kvcache(ref, name, *, b, h, hk, sq, sk, d, dtype, causal=False, local=True,
                 page=16, num_splits=2):
    """Recipe of test_flash_attn_kvcache (test.py:1355-1594), paged, no new KV, CPU, seed 0."""
    torch.random.manual_seed(0)
    window = (-1, -1) if not local else tuple(int(x) for x in torch.randint(0, sk, (2,)))
    q = torch.randn(b, sq, h, d, dtype=dtype)
    kc, vc, table, kp, vp, nblocks = ref["_generate_block_kvcache"](sk, page, b, hk, d, "cpu", dtype)
    cache_seqlens = torch.randint(1, sk + 1, (b,), dtype=torch.int32)
    kpm = torch.arange(sk).view(1, -1) < cache_seqlens.view(-1, 1)
    krep = kc.repeat_interleave(h // hk, dim=2)
    vrep = vc.repeat_interleave(h // hk, dim=2)
    out_ref, _ = ref["attention_ref"](q, krep, vrep, None, kpm, None, 0.0, None, causal=causal,
                                      window_size=window)
    out_pt, _ = ref["attention_ref"](q, krep, vrep, None, kpm, None, 0.0, None, causal=causal,
                                     window_size=window, upcast=False, reorder_ops=True)
    mine, _ = ours.attention_ref(q, kc, vc, None, kpm, None, 0.0, None, causal=causal,
                                 window_size=window)
    _same(mine, out_ref, name + ":out_ref")
    kp, vp, table, nblocks = _compact_pool(kp, vp, table, cache_seqlens, page)
    t = dict(q=q, k_cache_paged=kp, v_cache_paged=vp, block_table=table,
             cache_seqlens=cache_seqlens, out_ref=out_ref, out_pt=out_pt)
    meta = dict(kind="kvcache", b=b, h=h, hk=hk, sq=sq, sk=sk, d=d, page=page,
                num_blocks=nblocks, num_splits=num_splits, dtype=str(dtype).split(".")[-1],
                causal=causal, window=list(window),
                recipe="test.py:1355-1594 (test_flash_attn_kvcache), paged, CPU, manual_seed(0)")
    _save(name, t, meta, regen=("q",))


def _compact_pool(kp, vp, table, cache_seqlens, page):
    """Keep only the pages the block table actually reaches (the first ceil(len/page) entries
    of each row), renumbered through a seeded permutation so the table stays a random mapping;
    unreached entries point at page 0.  The outputs are unchanged (unreached keys are masked
    by cache_seqlens); the recipe's pool is 3x the reached pages (test.py:1605)."""
    used = []
    for bi in range(table.shape[0]):
        n = max(1, -(-int(cache_seqlens[bi]) // page))
        used += [int(x) for x in table[bi, :n]]
    perm = torch.randperm(len(used), generator=torch.Generator().manual_seed(11))
    new_id = {old: int(perm[i]) for i, old in enumerate(used)}
    order = sorted(new_id, key=new_id.get)
    kp2, vp2 = kp[order].clone(), vp[order].clone()
    t2 = torch.zeros_like(table)
    for bi in range(table.shape[0]):
        n = max(1, -(-int(cache_seqlens[bi]) // page))
        t2[bi, :n] = torch.tensor([new_id[int(x)] for x in table[bi, :n]], dtype=table.dtype)
    return kp2, vp2, t2, len(order)


def check_restatement_masks(ref):
    """construct_local_mask / padding-mask / paged-cache restatement KATs."""
    for (sq, sk, w) in [(5, 9, (-1, 0)), (7, 7, (2, 1)), (9, 4, (0, 3)), (3, 11, (-1, 2)),
                        (4, 6, (1, -1))]:
        _same(ours.local_mask(sq, sk, w), ref["construct_local_mask"](sq, sk, w), f"mask{sq},{sk},{w}")
    torch.manual_seed(3)
    kpm = ref["generate_random_padding_mask"](37, 3, "cpu", mode="random")
    qpm = ref["generate_random_padding_mask"](29, 3, "cpu", mode="third")
    for w in [(-1, 0), (4, 2), (0, 0)]:
        _same(ours.local_mask(29, 37, w, qpm, kpm), ref["construct_local_mask"](29, 37, w, qpm, kpm),
              f"padded-mask{w}")
    torch.manual_seed(5)
    a = ref["generate_random_padding_mask"](41, 4, "cpu", mode="random")
    torch.manual_seed(5)
    _same(ours.random_padding_mask(41, 4, "cpu", mode="random"), a, "random_padding_mask")
    torch.manual_seed(7)
    r = ref["_generate_block_kvcache"](50, 16, 2, 3, 8, "cpu", torch.float16)
    torch.manual_seed(7)
    m = ours.block_kvcache(50, 16, 2, 3, 8, "cpu", torch.float16)
    for x, y, nm in zip(m[:5], r[:5], ("kc", "vc", "table", "kp", "vp")):
        _same(x, y, "block_kvcache:" + nm)
    assert m[5] == r[5]
    slopes = torch.rand(2, 3) * 0.3
    _same(ours.alibi_bias(slopes, 7, 9, qpm[:2, :7], kpm[:2, :9]),
          ref["attn_bias_from_alibi_slopes"](slopes, 7, 9, qpm[:2, :7], kpm[:2, :9]), "alibi-padded")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check-only", action="store_true")
    args = ap.parse_args()
    ref = load_reference_oracle()
    check_restatement_masks(ref)
    save = not args.check_only
    f16, bf16 = torch.float16, torch.bfloat16
    if save:
        for fn in os.listdir(GOLDEN) if os.path.isdir(GOLDEN) else []:
            if fn.endswith(".safetensors"):
                os.remove(os.path.join(GOLDEN, fn))
    # C1 (BASELINE configs[0]): fp32 CPU plumbing case.
    case_fwd(ref, "c1_fwd_fp32_b1h4s128d64", b=1, h=4, hk=4, sq=128, sk=128, d=64,
             dtype=torch.float32, causal=False, grads=False, save=save)
    # The reference's one live fwd test point (test.py:711-750).
    case_fwd(ref, "fwd_f16_b1h1s128d128_causal", b=1, h=1, hk=1, sq=128, sk=128, d=128,
             dtype=f16, causal=True, save=save)
    # Widened upstream grid (commented lists at test.py:711-750), small sizes.
    case_fwd(ref, "fwd_bf16_b1h2s256d128_causal", b=1, h=2, hk=2, sq=256, sk=256, d=128,
             dtype=bf16, causal=True, save=save)
    case_fwd(ref, "fwd_bf16_b1h4hk2_q113k203_d128", b=1, h=4, hk=2, sq=113, sk=203, d=128,
             dtype=bf16, causal=False, save=save)
    case_fwd(ref, "fwd_f16_b1h4hk1_q203k113_d64_causal", b=1, h=4, hk=1, sq=203, sk=113, d=64,
             dtype=f16, causal=True, save=save)
    case_fwd(ref, "fwd_f16_b1h2_q108k256_d128_local", b=1, h=2, hk=2, sq=108, sk=256, d=128,
             dtype=f16, causal=False, local=True, save=save)
    case_fwd(ref, "fwd_f16_b1h2_q128k217_d80_alibi", b=1, h=2, hk=2, sq=128, sk=217, d=80,
             dtype=f16, causal=False, alibi=True, save=save)
    case_fwd(ref, "fwd_f16_b1h4_q64k96_d40_causal_alibi", b=1, h=4, hk=4, sq=64, sk=96, d=40,
             dtype=f16, causal=True, alibi=True, save=save)
    case_fwd(ref, "fwd_bf16_b1h4_q128k128_d64_softcap", b=1, h=4, hk=4, sq=128, sk=128, d=64,
             dtype=bf16, causal=True, softcap=50.0, save=save)
    case_fwd(ref, "fwd_f16_b2h6hk2_q1k147_d128", b=2, h=6, hk=2, sq=1, sk=147, d=128,
             dtype=f16, causal=False, grads=False, save=save)
    if save:
        # attention_ref's dropout branch (test.py:387-394)
        case_dropout(ref, "dropout_f16_b2h4hk2_q97k131_d64_causal", b=2, h=4, hk=2, sq=97,
                     sk=131, d=64, dtype=f16, causal=True, p_drop=0.17)
        # Varlen grid points (test.py:988-1025), downsized.
        case_varlen(ref, "varlen_f16_b4h3_q113k203_d64_causal", b=4, h=3, hk=3, sq=113, sk=203,
                    d=64, dtype=f16, causal=True)
        case_varlen(ref, "varlen_f16_b4h2hk1_q128k217_d128", b=4, h=2, hk=1, sq=128, sk=217,
                    d=128, dtype=f16, causal=False)
        case_varlen(ref, "varlen_f16_b4h6hk1_q1k147_d80_local", b=4, h=6, hk=1, sq=1, sk=147,
                    d=80, dtype=f16, causal=False, local=True)
        case_varlen(ref, "varlen_bf16_b4h6hk2_q108k256_d40_causal_local", b=4, h=6, hk=2, sq=108,
                    sk=256, d=40, dtype=bf16, causal=True, local=True)
        # Paged KV-cache grid points (test.py:1309-1353), downsized head counts kept.
        case_kvcache(ref, "kvcache_f16_b2h6_q1k128_mha", b=2, h=6, hk=6, sq=1, sk=128, d=128,
                     dtype=f16)
        case_kvcache(ref, "kvcache_f16_b2h6hk1_q1k339_mqa", b=2, h=6, hk=1, sq=1, sk=339, d=128,
                     dtype=f16)
        case_kvcache(ref, "kvcache_f16_b2h6hk1_q3k799_mqa", b=2, h=6, hk=1, sq=3, sk=799, d=128,
                     dtype=f16)
        case_kvcache(ref, "kvcache_f16_b2h6hk3_q64k256_gqa", b=2, h=6, hk=3, sq=64, sk=256,
                     d=128, dtype=f16)
    total = sum(os.path.getsize(os.path.join(GOLDEN, f)) for f in os.listdir(GOLDEN))
    print(f"golden fixtures OK ({total/1e6:.2f} MB); restatement matches reference bit for bit")


if __name__ == "__main__":
    main()

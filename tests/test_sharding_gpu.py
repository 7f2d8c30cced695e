"""GPU: sharding.py driving the HIP kernels.

A one-rank RCCL process group (the `nccl` backend on ROCm) on the box's GPU, so every sharded
entry runs its real path - shard selection, the gfx950 kernels on the rank's views (head-sliced
views through fmha_fwd_strided) - against the pinned CPU oracle with the reference's own rules
(test.py:975 forward 2x, :1593-1594 kvcache 3x + 1e-5).  At world size 1 no collective is
issued (all_gather_dim returns the local shard), so the RCCL all-gather itself is NOT exercised
here: the N > 1 partition / assembly / gradient logic is covered on CPU by
tests/test_sharding.py (gloo, world 2) and stays unmeasured on RCCL until a multi-GPU run.
"""
import os
import socket

import pytest
import torch

from oracle import attention_ref as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    yield dist
    dist.destroy_process_group()


def _check(got, q, k, v, mult=2.0, atol=0.0, **kw):
    ref, _ = orc.attention_ref(q, k, v, **kw)
    pt, _ = orc.attention_ref(q, k, v, upcast=False, reorder_ops=True, **kw)
    ok, err, bound = orc.parity_ok(got.cpu(), ref, pt, mult, atol)
    assert ok, f"max|out-ref| = {err:.3g} > {bound:.3g}"


@pytest.mark.parametrize("prefer", ["heads", "batch"])
def test_sharded_attention_hip(pg, prefer):
    from xf_flash_attention_cutlass_amd import sharding as sh
    g = torch.Generator().manual_seed(1)
    q = torch.randn(2, 700, 8, 128, generator=g).bfloat16()
    k = torch.randn(2, 700, 2, 128, generator=g).bfloat16()
    v = torch.randn(2, 700, 2, 128, generator=g).bfloat16()
    out, shard = sh.sharded_attention(q.to(DEV), k.to(DEV), v.to(DEV), prefer=prefer, causal=True)
    torch.cuda.synchronize()
    assert shard.size == (8 if prefer == "heads" else 2)
    _check(out, q, k, v, causal=True)


def test_sharded_varlen_hip(pg):
    from xf_flash_attention_cutlass_amd import sharding as sh
    lens = [300, 1, 777, 64, 1025]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    g = torch.Generator().manual_seed(2)
    q = torch.randn(int(cu[-1]), 4, 128, generator=g).bfloat16()
    k = torch.randn(int(cu[-1]), 4, 128, generator=g).bfloat16()
    v = torch.randn(int(cu[-1]), 4, 128, generator=g).bfloat16()
    out, idx = sh.sharded_varlen(q.to(DEV), k.to(DEV), v.to(DEV), cu.to(DEV), cu.to(DEV), causal=True)
    torch.cuda.synchronize()
    assert idx.numel() == int(cu[-1])
    for i in range(len(lens)):
        a, b = int(cu[i]), int(cu[i + 1])
        _check(out[a:b][None], q[a:b][None], k[a:b][None], v[a:b][None], causal=True)


def test_sharded_decode_hip(pg):
    from xf_flash_attention_cutlass_amd import sharding as sh
    b, hk, h, d, page, sk = 5, 2, 8, 128, 16, 333
    kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(3)
    qd = torch.randn(b, 1, h, d, generator=g).bfloat16()
    seqlens = torch.tensor([333, 17, 1, 200, 64], dtype=torch.int32)
    out, bs = sh.sharded_decode(qd.to(DEV), kp.to(DEV), vp.to(DEV), seqlens.to(DEV), table.to(DEV))
    torch.cuda.synchronize()
    assert bs.size == b
    for i in range(b):
        n = int(seqlens[i])
        idx = table[i].long()
        kk = kp[idx].reshape(1, -1, hk, d)[:, :n]
        vv = vp[idx].reshape(1, -1, hk, d)[:, :n]
        _check(out[i:i + 1], qd[i:i + 1], kk, vv, mult=3.0, atol=1e-5)


def test_sharded_backward_hip(pg):
    """Backward through sharded_attention and sharded_varlen on the HIP kernels (one-rank
    group: the gathers' backward is the identity there; the N > 1 narrow is covered by the gloo
    world-2 test).  Gradients against oracle autograd with the reference's rule (3x + 1e-5,
    test.py:984-986)."""
    from xf_flash_attention_cutlass_amd import sharding as sh
    g = torch.Generator().manual_seed(4)
    q = torch.randn(2, 300, 8, 128, generator=g).bfloat16()
    k = torch.randn(2, 300, 2, 128, generator=g).bfloat16()
    v = torch.randn(2, 300, 2, 128, generator=g).bfloat16()
    do = torch.randn(2, 300, 8, 128, generator=g).bfloat16()
    qd, kd, vd = (x.to(DEV).requires_grad_(True) for x in (q, k, v))
    out, _ = sh.sharded_attention(qd, kd, vd, causal=True)
    got = torch.autograd.grad(out, (qd, kd, vd), do.to(DEV))
    ref, pt = [], []
    for up, dst in ((True, ref), (False, pt)):
        qq, kk, vv = (x.clone().requires_grad_(True) for x in (q, k, v))
        o, _ = orc.attention_ref(qq, kk, vv, causal=True, upcast=up, reorder_ops=not up)
        dst.extend(torch.autograd.grad(o, (qq, kk, vv), do))
    for x, r, p in zip(got, ref, pt):
        ok, err, bound = orc.parity_ok(x.cpu(), r, p, 3.0, 1e-5)
        assert ok, f"sharded dense grad: {err:.3g} > {bound:.3g}"

    lens = [300, 1, 250, 64]
    n = sum(lens)
    qv = torch.randn(n, 4, 128, generator=g).bfloat16()
    kv_ = torch.randn(n, 4, 128, generator=g).bfloat16()
    vv_ = torch.randn(n, 4, 128, generator=g).bfloat16()
    dov = torch.randn(n, 4, 128, generator=g).bfloat16()
    plan = sh.varlen_plan(lens, lens, 1, 0, DEV)
    qd, kd, vd = (x.to(DEV).requires_grad_(True) for x in (qv, kv_, vv_))
    out, _ = sh.sharded_varlen(qd, kd, vd, plan=plan, causal=True)
    got = torch.autograd.grad(out, (qd, kd, vd), dov.to(DEV))
    cu = [0]
    for x in lens:
        cu.append(cu[-1] + x)
    for i in range(len(lens)):
        a, b = cu[i], cu[i + 1]
        ref, pt = [], []
        for up, dst in ((True, ref), (False, pt)):
            qq, kk, vv = (x[a:b][None].clone().requires_grad_(True) for x in (qv, kv_, vv_))
            o, _ = orc.attention_ref(qq, kk, vv, causal=True, upcast=up, reorder_ops=not up)
            dst.extend(torch.autograd.grad(o, (qq, kk, vv), dov[a:b][None]))
        for x, r, p in zip(got, ref, pt):
            ok, err, bound = orc.parity_ok(x[a:b][None].cpu(), r, p, 3.0, 1e-5)
            assert ok, f"sharded varlen grad seq {i}: {err:.3g} > {bound:.3g}"

"""CPU: multi-GPU sharding logic with a world-size-2 gloo process group.

The per-rank compute is injected (`local_fn`), so these tests exercise exactly the
partitioning and the all-gather assembly the GPU path uses (RCCL over xGMI there), with the
CPU oracle standing in as the per-shard compute — as a checker, never as the product path.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from xf_flash_attention_cutlass_amd import sharding as sh


def test_even_ranges():
    assert [s.size for s in sh.even_ranges(10, 4)] == [3, 3, 2, 2]
    assert sh.even_ranges(3, 3)[-1] == sh.Shard(2, 3)


def test_head_shards_are_gqa_aligned():
    shards = sh.head_shards(32, 8, 8)
    assert all(q.size == 4 and k.size == 1 for q, k in shards)
    assert [q.start for q, _ in shards] == list(range(0, 32, 4))
    shards = sh.head_shards(12, 6, 4)        # uneven: 2,2,1,1 kv heads
    assert [k.size for _, k in shards] == [2, 2, 1, 1]
    assert all(q.start == k.start * 2 and q.stop == k.stop * 2 for q, k in shards)
    with pytest.raises(ValueError):
        sh.head_shards(32, 2, 8)


def test_balanced_sequences_cover_and_balance():
    lq = [1024, 7168, 3000, 64, 5000, 2048, 4096, 1]
    parts = sh.balanced_sequences(lq, lq, 4)
    assert sorted(i for p in parts for i in p) == list(range(len(lq)))
    loads = [sum(lq[i] ** 2 for i in p) for p in parts]
    assert max(loads) <= 7168 ** 2 + 1   # the largest sequence bounds the max load here


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, kind, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import attention_ref as orc
        torch.manual_seed(0)   # identical (replicated) inputs on every rank
        if kind == "heads":
            x = torch.randn(2, 40, 8, 16)
            k = torch.randn(2, 40, 4, 16)
            v = torch.randn(2, 40, 4, 16)

            def local(qq, kk, vv, causal=False):
                return orc.attention_ref(qq, kk, vv, causal=causal)[0]
            out, _ = sh.sharded_attention(x, k, v, local_fn=local, causal=True)
            ref = local(x, k, v, causal=True)
            ok = torch.allclose(out, ref, atol=1e-6)
        elif kind == "heads_uneven":
            # 3 kv heads over 2 ranks: query heads 4 / 2 gathered along dim 2 with padding
            x = torch.randn(2, 30, 6, 16)
            k = torch.randn(2, 30, 3, 16)
            v = torch.randn(2, 30, 3, 16)

            def local(qq, kk, vv, causal=False):
                return orc.attention_ref(qq, kk, vv, causal=causal)[0]
            out, qs = sh.sharded_attention(x, k, v, local_fn=local, causal=True)
            ref = local(x, k, v, causal=True)
            ok = torch.allclose(out, ref, atol=1e-6) and qs.size == (4 if rank == 0 else 2)
        elif kind == "heads_alibi":
            x = torch.randn(2, 24, 8, 16)
            k = torch.randn(2, 24, 4, 16)
            v = torch.randn(2, 24, 4, 16)
            slopes = torch.rand(2, 8)

            def local(qq, kk, vv, causal=False, alibi_slopes=None):
                bias = orc.alibi_bias(alibi_slopes, qq.shape[1], kk.shape[1], causal=causal)
                return orc.attention_ref(qq, kk, vv, attn_bias=bias, causal=causal)[0]
            out, qs = sh.sharded_attention(x, k, v, local_fn=local, causal=True,
                                           alibi_slopes=slopes)
            ref = local(x, k, v, causal=True, alibi_slopes=slopes)
            ok = torch.allclose(out, ref, atol=1e-6) and qs.size == 4
        elif kind == "batch":
            # fewer kv heads than ranks: batch shards (uneven: 3 rows over 2 ranks)
            x = torch.randn(3, 20, 2, 16)
            k = torch.randn(3, 20, 1, 16)
            v = torch.randn(3, 20, 1, 16)
            slopes = torch.rand(3, 2)

            def local(qq, kk, vv, causal=False, alibi_slopes=None):
                bias = orc.alibi_bias(alibi_slopes, qq.shape[1], kk.shape[1], causal=causal)
                return orc.attention_ref(qq, kk, vv, attn_bias=bias, causal=causal)[0]
            out, bs = sh.sharded_attention(x, k, v, local_fn=local, causal=True,
                                           alibi_slopes=slopes)
            ref = local(x, k, v, causal=True, alibi_slopes=slopes)
            ok = torch.allclose(out, ref, atol=1e-6) and bs.size == (2 if rank == 0 else 1)
        elif kind == "batch_pref":
            # prefer="batch" with a batch the world divides: batch shards although the kv heads
            # would split (the gather along dim 0 needs no copy)
            x = torch.randn(4, 24, 8, 16)
            k = torch.randn(4, 24, 4, 16)
            v = torch.randn(4, 24, 4, 16)

            def local(qq, kk, vv, causal=False):
                return orc.attention_ref(qq, kk, vv, causal=causal)[0]
            out, bs = sh.sharded_attention(x, k, v, local_fn=local, causal=True, prefer="batch")
            ref = local(x, k, v, causal=True)
            ok = torch.allclose(out, ref, atol=1e-6) and bs.size == 2
        elif kind == "decode":
            # C5 assembly: batch-sharded paged decode, pages stay in the shared pool
            b, hk, h, d, page, sk = 5, 2, 8, 16, 4, 37
            kc, vc, table, kp, vp, _ = orc.block_kvcache(sk, page, b, hk, d, dtype=torch.float32)
            qd = torch.randn(b, 1, h, d)
            seqlens = torch.tensor([37, 5, 1, 20, 36], dtype=torch.int32)

            def local(qq, kpool, vpool, sl, bt):
                outs = []
                for i in range(qq.shape[0]):
                    n = int(sl[i])
                    idx = bt[i].long()
                    kk = kpool[idx].reshape(1, -1, hk, d)[:, :n]
                    vv = vpool[idx].reshape(1, -1, hk, d)[:, :n]
                    outs.append(orc.attention_ref(qq[i:i + 1], kk, vv)[0])
                return torch.cat(outs)
            out, bs = sh.sharded_decode(qd, kp, vp, seqlens, table, local_fn=local)
            ref = local(qd, kp, vp, seqlens, table)
            ok = torch.allclose(out, ref, atol=1e-6) and bs.size == (3 if rank == 0 else 2)
        else:
            lens = [5, 17, 1, 30, 9]
            cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
            x = torch.randn(int(cu[-1]), 4, 16)
            k = torch.randn(int(cu[-1]), 2, 16)
            v = torch.randn(int(cu[-1]), 2, 16)

            def local(qq, kk, vv, cq, ck, mq, mk, causal=False):
                outs = []
                for i in range(len(cq) - 1):
                    a, b = int(cq[i]), int(cq[i + 1])
                    c, d = int(ck[i]), int(ck[i + 1])
                    outs.append(orc.attention_ref(qq[a:b][None], kk[c:d][None], vv[c:d][None],
                                                  causal=causal)[0][0])
                return torch.cat(outs)
            out, _ = sh.sharded_varlen(x, k, v, cu, cu, local_fn=local, causal=True)
            ref = local(x, k, v, cu, cu, max(lens), max(lens), causal=True)
            ok = torch.allclose(out, ref, atol=1e-6)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _grad_worker(rank, world, port, kind, q):
    """Backward through the sharded paths: every rank computes the same loss from the gathered
    output; the all-gathers' backward narrows the gradient to the rank's shard, so the ranks'
    gradients of the replicated q / k / v, summed, are the unsharded gradients."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import attention_ref as orc
        torch.manual_seed(0)
        if kind == "varlen":
            lens = [5, 17, 1, 30, 9]
            n = sum(lens)
            x, k, v = torch.randn(n, 4, 16), torch.randn(n, 2, 16), torch.randn(n, 2, 16)

            def local(qq, kk, vv, cq, ck, mq, mk, causal=False):
                outs = []
                for i in range(len(cq) - 1):
                    a, b = int(cq[i]), int(cq[i + 1])
                    c, d = int(ck[i]), int(ck[i + 1])
                    outs.append(orc.attention_ref(qq[a:b][None], kk[c:d][None], vv[c:d][None],
                                                  causal=causal)[0][0])
                return torch.cat(outs)
            plan = sh.varlen_plan(lens, lens, world, rank, "cpu")   # host lengths: no sync
            cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)

            def run(a, b, c, sharded):
                if sharded:
                    return sh.sharded_varlen(a, b, c, local_fn=local, plan=plan, causal=True)[0]
                return local(a, b, c, cu, cu, max(lens), max(lens), causal=True)
        else:
            shapes = {"heads": ((2, 24, 8, 16), 4), "heads_uneven": ((2, 20, 6, 16), 3),
                      "batch": ((3, 20, 2, 16), 1)}
            (b, s_, h, d), hk = shapes[kind]
            x, k, v = torch.randn(b, s_, h, d), torch.randn(b, s_, hk, d), torch.randn(b, s_, hk, d)

            def local(qq, kk, vv, causal=False):
                return orc.attention_ref(qq, kk, vv, causal=causal)[0]

            def run(a, b_, c, sharded):
                if sharded:
                    return sh.sharded_attention(a, b_, c, local_fn=local, causal=True)[0]
                return local(a, b_, c, causal=True)
        w = torch.randn(x.shape[:-1] + (v.shape[-1],))
        grads = []
        for sharded in (True, False):
            xs, ks, vs = (t.clone().requires_grad_(True) for t in (x, k, v))
            out = run(xs, ks, vs, sharded)
            (out * w).sum().backward()
            grads.append([t.grad for t in (xs, ks, vs)])
        ok = True
        for gs, gr in zip(*grads):
            dist.all_reduce(gs)          # each rank holds its shard's part; the sum is the whole
            ok = ok and torch.allclose(gs, gr, atol=1e-5)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _spawn(target, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    return dict(q.get(timeout=5) for _ in range(2))


@pytest.mark.parametrize("kind", ["heads", "heads_uneven", "batch", "varlen"])
def test_sharded_backward_world2_gloo(kind):
    assert _spawn(_grad_worker, kind) == {0: True, 1: True}


def test_varlen_plan_host_only():
    """The plan is built from host lengths alone; the scatter index covers every packed token
    once and each rank's positions are its sequences'."""
    lens = [300, 1, 777, 64, 1025]
    plans = [sh.varlen_plan(lens, lens, 2, r, "cpu") for r in range(2)]
    nmax = max(plans[0].counts)
    assert sorted(plans[0].inv.tolist()) == sorted(
        r * nmax + j for r in range(2) for j in range(plans[0].counts[r]))
    assert sorted(plans[0].mine_q.tolist() + plans[1].mine_q.tolist()) == list(range(sum(lens)))
    assert plans[0].cu_q[-1].item() == plans[0].counts[0]


@pytest.mark.parametrize("kind", ["heads", "heads_uneven", "heads_alibi", "batch", "batch_pref",
                                  "decode", "varlen"])
def test_sharded_world2_gloo(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}

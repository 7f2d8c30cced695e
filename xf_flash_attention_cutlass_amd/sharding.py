"""Multi-GPU sharding of the attention hot path (one process per GPU, torch.distributed).

The reference has no distributed code (no NCCL/RCCL call sites).  Attention has
no reduction across (batch, head) units in the forward, so the units are partitioned across
ranks and every rank runs the single-GPU kernels on its shard with NO collective in the data
path; the only exchange is an optional all-gather (RCCL over xGMI on MI355X, `nccl` backend =
RCCL) that assembles the sharded outputs on every rank:

  * dense fwd/bwd (C2/C3)  : shard heads in contiguous, GQA-aligned ranges (a K/V head and all
                             query heads that read it stay on one rank, so dK/dV need no
                             cross-rank reduction); batch shards when there are fewer kv heads
                             than ranks (then every rank needs at least one batch element);
  * varlen (C4)            : shard whole sequences, greedy-balanced on sum(s_q * s_k);
  * paged decode (C5)      : shard the batch; every rank owns its sequences' pages, no KV moves.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Sequence, Tuple

import torch


@dataclass(frozen=True)
class Shard:
    start: int
    stop: int

    @property
    def size(self) -> int:
        return self.stop - self.start


def even_ranges(n: int, world: int) -> List[Shard]:
    """Split range(n) into `world` contiguous chunks whose sizes differ by at most one."""
    base, rem = divmod(n, world)
    out, s = [], 0
    for r in range(world):
        e = s + base + (1 if r < rem else 0)
        out.append(Shard(s, e))
        s = e
    return out


def head_shards(num_heads: int, num_heads_k: int, world: int) -> List[Tuple[Shard, Shard]]:
    """GQA-aligned head ranges: rank r gets kv heads [a, b) and query heads [a*G, b*G)."""
    if num_heads % num_heads_k:
        raise ValueError("num_heads must be a multiple of num_heads_k")
    if num_heads_k < world:
        raise ValueError(f"cannot shard {num_heads_k} kv heads over {world} ranks; use batch shards")
    g = num_heads // num_heads_k
    return [(Shard(s.start * g, s.stop * g), s) for s in even_ranges(num_heads_k, world)]


def balanced_sequences(seqlens_q: Sequence[int], seqlens_k: Sequence[int], world: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment of whole sequences on cost s_q * s_k."""
    cost = [int(a) * int(b) for a, b in zip(seqlens_q, seqlens_k)]
    order = sorted(range(len(cost)), key=lambda i: -cost[i])
    load = [0] * world
    parts: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda j: (load[j], j))
        parts[r].append(i)
        load[r] += cost[i]
    return [sorted(p) for p in parts]


def _world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


def all_gather_heads(local: torch.Tensor, shards: List[Tuple[Shard, Shard]], head_dim: int = 2):
    """Assemble [b, s, H, d] from per-rank head shards [b, s, H_r, d] (all ranks get the full
    tensor)."""
    return all_gather_dim(local, [q.size for q, _ in shards], head_dim)


def _slice_alibi(alibi, heads: Shard | None = None, batch: Shard | None = None):
    """ALiBi slopes ([H] or [b, H]) restricted to a rank's query heads / batch rows."""
    if alibi is None:
        return None
    if heads is not None:
        alibi = alibi[..., heads.start:heads.stop]
    if batch is not None and alibi.dim() == 2:
        alibi = alibi[batch.start:batch.stop]
    return alibi.contiguous()


def _gather_dim_impl(local: torch.Tensor, sizes: Sequence[int], dim: int, dist, world: int):
    """The collective itself (world > 1).  Even shards: along dim 0 one all_gather_into_tensor
    whose rank-major buffer IS the result; along another dim (head shards) the rank-major
    buffer is moved to `dim` with one copy.  Uneven shards pad to the largest piece along `dim`
    and drop the padding afterwards."""
    local = local.contiguous()
    nmax = max(sizes)
    shape = list(local.shape)
    if min(sizes) == nmax:
        gathered = local.new_empty([world * shape[0]] + shape[1:])   # rank-major along dim 0
        dist.all_gather_into_tensor(gathered, local)
        if dim == 0:
            return gathered
        # [world, *shape] -> pieces side by side along dim
        g = gathered.view([world] + shape).movedim(0, dim)
        return g.reshape(shape[:dim] + [world * nmax] + shape[dim + 1:])
    shape[dim] = nmax
    buf = local.new_zeros(shape)
    buf.narrow(dim, 0, local.shape[dim]).copy_(local)
    gathered = local.new_empty([world * shape[0]] + shape[1:])
    dist.all_gather_into_tensor(gathered, buf)
    gathered = gathered.view([world] + shape)
    return torch.cat([gathered[r].narrow(dim, 0, sizes[r]) for r in range(world)], dim=dim)


class _AllGatherDim(torch.autograd.Function):
    """All-gather along `dim` whose backward hands each rank the gradient of its own piece.

    Every rank holds the whole gathered output and (data-parallel replicas of one step) computes
    the same loss from it, so d loss / d (my piece) is the slice of d loss / d out at my offset:
    the backward is a narrow, with no communication."""

    @staticmethod
    def forward(ctx, local, sizes, dim, rank):
        dist, _, world = _world()
        ctx.dim, ctx.start, ctx.size = dim, sum(sizes[:rank]), sizes[rank]
        return _gather_dim_impl(local, sizes, dim, dist, world)

    @staticmethod
    def backward(ctx, grad):
        return grad.narrow(ctx.dim, ctx.start, ctx.size), None, None, None


def all_gather_dim(local: torch.Tensor, sizes: Sequence[int], dim: int):
    """Concatenate per-rank pieces along `dim` (rank r holds sizes[r] entries) on every rank.
    Differentiable (`_AllGatherDim`): the backward narrows the output gradient to this rank's
    piece.  World size 1 runs no collective: the local piece is the result."""
    dist, rank, world = _world()
    if world == 1:
        return local
    return _AllGatherDim.apply(local, list(sizes), dim, rank)


def sharded_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                      local_fn: Callable | None = None, gather: bool = True,
                      prefer: str = "heads", **kw):
    """Dense attention sharded over ranks: every rank holds the full (replicated) q/k/v views,
    computes its GQA-aligned query-head range with `local_fn` (default: the gfx950 kernels)
    and, if `gather`, all-gathers the outputs.  With fewer kv heads than ranks, or with
    prefer="batch" and a batch the world divides (whose gather along dim 0 needs no copy), the
    batch is sharded instead.  ALiBi slopes in `kw` are sliced to the rank's heads / batch rows.
    Returns (out, my shard): a query-head range or a batch range (see `attention_shards`)."""
    dist, rank, world = _world()
    if local_fn is None:
        from . import flash_attn_func as local_fn
    kind, shards = attention_shards(q.shape[0], q.shape[2], k.shape[2], world, prefer)
    alibi = kw.pop("alibi_slopes", None)
    if kind == "heads":
        qs, ks = shards[rank]
        if alibi is not None:
            kw["alibi_slopes"] = _slice_alibi(alibi, heads=qs)
        # head-sliced views go to the kernels as they are (fmha_fwd_strided): no copies
        out_local = local_fn(q[:, :, qs.start:qs.stop], k[:, :, ks.start:ks.stop],
                             v[:, :, ks.start:ks.stop], **kw)
        if not gather:
            return out_local, qs
        return all_gather_dim(out_local, [a.size for a, _ in shards], 2), qs
    bs = shards[rank]
    if alibi is not None:
        kw["alibi_slopes"] = _slice_alibi(alibi, batch=bs)
    out_local = local_fn(q[bs.start:bs.stop], k[bs.start:bs.stop], v[bs.start:bs.stop], **kw)
    if not gather:
        return out_local, bs
    return all_gather_dim(out_local, [s.size for s in shards], 0), bs


def attention_shards(batch: int, num_heads: int, num_heads_k: int, world: int,
                     prefer: str = "heads"):
    """("heads", [(q heads, kv heads)] per rank) when every rank gets at least one kv head
    (unless prefer="batch" and world divides the batch), else ("batch", [batch range] per
    rank)."""
    if prefer not in ("heads", "batch"):
        raise ValueError(f"prefer must be 'heads' or 'batch' (got {prefer!r})")
    if prefer == "batch" and batch % world == 0:
        return "batch", batch_shards(batch, world)
    if num_heads_k >= world:
        return "heads", head_shards(num_heads, num_heads_k, world)
    if batch < world:
        raise ValueError(f"cannot shard {num_heads_k} kv heads or {batch} batch rows over {world} ranks")
    return "batch", batch_shards(batch, world)


@dataclass(frozen=True)
class VarlenPlan:
    """Sequence shards of one packed varlen batch, built once from HOST-side lengths (no device
    sync when it is reused): every rank can compute every rank's part, so the per-rank token
    counts need no exchange.

    mine_q / mine_k : packed positions of this rank's query / key tokens (device, int64)
    cu_q / cu_k     : this rank's local cumulative lengths (device, int32)
    max_q / max_k   : this rank's longest sequences (0 if it has none)
    counts          : query tokens per rank;  inv: for each packed query position, its row in the
                      rank-major gathered [world * max(counts)] buffer (device, int64)"""
    parts: tuple
    mine_q: torch.Tensor
    mine_k: torch.Tensor
    cu_q: torch.Tensor
    cu_k: torch.Tensor
    max_q: int
    max_k: int
    counts: tuple
    inv: torch.Tensor


def varlen_plan(seqlens_q: Sequence[int], seqlens_k: Sequence[int], world: int, rank: int,
                device) -> VarlenPlan:
    """Plan for `sharded_varlen` from host lengths (lists of ints), balanced on s_q * s_k."""
    lq = [int(x) for x in seqlens_q]
    lk = [int(x) for x in seqlens_k]
    parts = balanced_sequences(lq, lk, world)
    cq = [0]
    ck = [0]
    for a, b in zip(lq, lk):
        cq.append(cq[-1] + a)
        ck.append(ck[-1] + b)

    def positions(seqs, cu):
        return [t for i in seqs for t in range(cu[i], cu[i + 1])]
    counts = [sum(lq[i] for i in p) for p in parts]
    nmax = max(counts) if counts else 0
    inv = [0] * cq[-1]
    for r, p in enumerate(parts):
        for j, t in enumerate(positions(p, cq)):
            inv[t] = r * nmax + j
    mine = parts[rank]

    def cum(lens):
        out = [0]
        for x in lens:
            out.append(out[-1] + x)
        return out
    L = lambda xs: torch.tensor(xs, dtype=torch.long, device=device)  # noqa: E731
    return VarlenPlan(
        parts=tuple(tuple(p) for p in parts),
        mine_q=L(positions(mine, cq)), mine_k=L(positions(mine, ck)),
        cu_q=torch.tensor(cum([lq[i] for i in mine]), dtype=torch.int32, device=device),
        cu_k=torch.tensor(cum([lk[i] for i in mine]), dtype=torch.int32, device=device),
        max_q=max([lq[i] for i in mine], default=0), max_k=max([lk[i] for i in mine], default=0),
        counts=tuple(counts), inv=L(inv))


class _GatherPacked(torch.autograd.Function):
    """All-gather of per-rank packed outputs back into the global packed order (rank-major
    buffer padded to the largest count, then one index_select).  Backward: this rank's rows of
    the output gradient, no communication (as `_AllGatherDim`)."""

    @staticmethod
    def forward(ctx, local, plan):
        dist, rank, world = _world()
        ctx.mine = plan.mine_q
        nmax = max(plan.counts)
        buf = local.new_zeros((nmax,) + tuple(local.shape[1:]))
        buf[: local.shape[0]] = local
        gathered = local.new_empty((world * nmax,) + tuple(local.shape[1:]))
        dist.all_gather_into_tensor(gathered, buf)
        return gathered.index_select(0, plan.inv)

    @staticmethod
    def backward(ctx, grad):
        return grad.index_select(0, ctx.mine), None


def sharded_varlen(q, k, v, cu_seqlens_q=None, cu_seqlens_k=None, local_fn: Callable | None = None,
                   gather: bool = True, plan: VarlenPlan | None = None, **kw):
    """Sequence-sharded varlen attention (C4): ranks take whole sequences, balanced on
    s_q*s_k; outputs are all-gathered back into the packed [total_q, H, d] order.  Pass a
    `plan` (`varlen_plan`, from host-side lengths) to run without any device sync; without
    one it is built from `cu_seqlens_*` (one host copy of each).  Differentiable: gradients
    flow to this rank's tokens of q / k / v.  Returns (out, packed positions of my tokens)."""
    dist, rank, world = _world()
    if local_fn is None:
        from . import flash_attn_varlen_func as local_fn
    if plan is None:
        cq = [int(x) for x in cu_seqlens_q.tolist()]
        ck = [int(x) for x in cu_seqlens_k.tolist()]
        plan = varlen_plan([b - a for a, b in zip(cq[:-1], cq[1:])],
                           [b - a for a, b in zip(ck[:-1], ck[1:])], world, rank, q.device)
    if plan.mine_q.numel():
        out_local = local_fn(q.index_select(0, plan.mine_q), k.index_select(0, plan.mine_k),
                             v.index_select(0, plan.mine_k), plan.cu_q, plan.cu_k, plan.max_q,
                             plan.max_k, **kw)
    else:
        # no sequences on this rank: a zero-row output still tied to q for autograd
        out_local = q.narrow(0, 0, 0) * 0
    if not gather or world == 1:
        return out_local, plan.mine_q
    return _GatherPacked.apply(out_local, plan), plan.mine_q


def batch_shards(batch: int, world: int) -> List[Shard]:
    """Paged decode (C5): contiguous batch ranges; each rank owns its sequences' KV pages."""
    return even_ranges(batch, world)


def sharded_decode(q: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor,
                   cache_seqlens: torch.Tensor, block_table: torch.Tensor,
                   local_fn: Callable | None = None, gather: bool = True, **kw):
    """Batch-sharded paged decode (C5): rank r takes batch rows `batch_shards(b, world)[r]` of
    q / cache_seqlens / block_table; the page pools stay where they are (a rank only reads the
    pages its own rows point to, so in a deployment each rank holds just its sequences'
    pages).  Outputs [b, sq, H, d] are all-gathered in batch order.  Returns (out, my rows)."""
    dist, rank, world = _world()
    if local_fn is None:
        from . import flash_attn_with_kvcache

        def local_fn(qq, kc, vc, sl, bt, **kk):
            return flash_attn_with_kvcache(qq, kc, vc, cache_seqlens=sl, block_table=bt, **kk)
    shards = batch_shards(q.shape[0], world)
    bs = shards[rank]
    alibi = kw.pop("alibi_slopes", None)
    if alibi is not None:
        kw["alibi_slopes"] = _slice_alibi(alibi, batch=bs)
    out_local = local_fn(q[bs.start:bs.stop].contiguous(), kcache, vcache,
                         cache_seqlens[bs.start:bs.stop].contiguous(),
                         block_table[bs.start:bs.stop].contiguous(), **kw)
    if not gather:
        return out_local, bs
    return all_gather_dim(out_local, [s.size for s in shards], 0), bs

"""Benchmark of the hot path on MI355X (BASELINE.json metric: attention TFLOPS/GPU).

Workloads (BASELINE.json configs):
  --mode fwd     (default) C2: mha_fwd B=4 H=32 S=4096 D=128 bf16 causal; one step = one
                 forward over the batch.  The default line also carries driver-timed
                 sub-results for C3 ("fwd_bwd"), C4 ("varlen"), C5 ("decode", full caches, and
                 "decode_ragged", cache lengths U[1, 32768]) and the fp8 forward, each with its
                 own roofline and CPU baseline (median of 3 runs), because the metric names fwd
                 and fwd+bwd and BASELINE lists all.
  --mode fwdbwd  C3: mha_fwd + mha_bwd, same shape (FLOPs = 3.5 x fwd, the usual convention).
  --mode varlen  C4: mha_varlen_fwd, 32 ragged sequences, total 131072 tokens, H=32 D=128 bf16.
  --mode decode  C5: paged-KV decode (fwd_kvcache), per GPU B=8 H=32 Hk=8 Sq=1, cache 32768
                 tokens, page 16, fp8 e4m3fn K/V; HBM-bound, reported in GB/s.
  --mode fwd_fp8 the C2 shape with fp8 e4m3fn Q/K/V (per-tensor descales) on the fp8 MFMA
                 (north_star's fp8 GEMMs; an extension, priced against the 5 PF fp8 peak).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode ...] [--scaling weak|strong]

Multi-GPU (one process per GPU, RCCL = torch.distributed "nccl" over xGMI).  With --gpus N > 1
and no WORLD_SIZE in the environment this process is only a launcher: before touching the GPU
it starts `python -m torch.distributed.run --nproc-per-node N` on this same file as a CHILD
process and exits with its status (the driver may also launch the ranks itself).  Sharding
(sharding.py; attention has no cross-unit reduction in the forward, so no collective sits in
the timed step):
  --scaling weak   (default) every rank owns a batch shard of the same per-GPU size: the global
                   batch is N x the single-GPU config (C2/C3: 4N sequences, C4: 32N sequences,
                   C5: 8N sequences, each rank holding its own sequences' pages);
  --scaling strong the global problem is the single-GPU config (C5: the survey's global B=64):
                   C2/C3 shard GQA-aligned head ranges (H/N heads per rank), C4 whole sequences
                   balanced on sum(s^2), C5 batch rows (64/N per rank).
The RCCL all-gather that assembles the sharded output on every rank is timed separately
("allgather", with "value_with_gather").  value = units processed by ALL ranks / max-over-ranks
wall time of exactly K steps between barriers.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0       # dense fp8 (block-scaled 32x32x64) MFMA peak
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md §HBM)
METRIC = "attention TFLOPS/GPU (fwd, fwd+bwd) at S=4096 D=128; % MI355X MFMA peak"


def fwd_flops(b, h, sq, sk, d, causal):
    f = 4.0 * b * h * sq * sk * d
    return f / 2 if causal else f


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["fwd", "fwdbwd", "varlen", "decode", "fwd_fp8"],
                    default="fwd")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--batch", type=int, default=0, help="default: 4 (fwd), 8 (decode)")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--seqlen", type=int, default=0, help="default: 4096 (fwd), 32768 (decode)")
    ap.add_argument("--headdim", type=int, default=128)
    ap.add_argument("--no-causal", action="store_true")
    ap.add_argument("--alibi", action="store_true",
                    help="fwd/fwdbwd: ALiBi slopes 2^(-8 (h+1) / H) (the standard geometric set)")
    ap.add_argument("--window-left", type=int, default=-1,
                    help="fwd/fwdbwd: left window (causal + wl = a sliding window of wl + 1 keys)")
    ap.add_argument("--ragged", action="store_true", help="decode: cache lengths U[1, S]")
    ap.add_argument("--page", type=int, default=0,
                    help="fwd: K/V in a paged cache of this page size (random-permutation block "
                         "table; the reference's fmha_page_kvcache_fwd prefill)")
    ap.add_argument("--rotate", type=int, default=0,
                    help="input sets cycled step by step (default: 2 for fwd/fwdbwd, so every "
                         "step reads inputs last touched two steps ago; C4/C5 inputs exceed the "
                         "256 MiB Infinity Cache on their own)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=6.0,
                    help="CPU budget per baseline (split over 3 runs; the median is reported)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the C3/C4/C5 sub-results of the default (fwd) line")
    ap.add_argument("--graph", choices=["on", "off"], default="off",
                    help="replay one step as a captured hipGraph")
    ap.add_argument("--opt", action="append", default=[],
                    help="name=value schedule knob (fmha_set_option) for A/B runs; recorded in "
                         "the line")
    ap.add_argument("--prewarm-s", type=float, default=1.0,
                    help="untimed seconds of steps before the warmup (GPU clock ramp)")
    ap.add_argument("--no-monitor", action="store_true",
                    help="do not sample the GPU clock / power (tools/gpu_monitor.py)")
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="launcher/aggregation self-test on CPU (gloo, a tiny matmul step): "
                         "NOT a benchmark; used by tests/test_bench_launcher.py")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- host info
def _threads():
    t = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    torch.set_num_threads(t)
    return t


def _host():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _median_runs(run, reps, budget_s):
    """`reps` timed runs of `run(budget)` (each returns (units, seconds, sample)), the median
    rate and every run's rate (median of >= 3 runs)."""
    rates, sample = [], ""
    for _ in range(reps):
        units, el, sample = run(budget_s / reps)
        rates.append(units / el)
    rates.sort()
    return rates[len(rates) // 2], rates, sample


def cpu_baseline_dense(heads: int, s: int, d: int, causal: bool, budget_s: float,
                       backward: bool = False, reps: int = 3):
    """Reference CPU eager path (oracle restatement of test.py:310-397, fp32 upcast; with
    `backward` also its autograd backward, FLOPs 3.5 x fwd as the GPU line counts) timed on
    the host cores: `reps` runs over a bounded sample of repeated (1 batch x `heads` heads)
    chunks of the same workload; the median run in TFLOP/s."""
    from oracle import attention_ref as orc
    threads = _threads()
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(1, s, heads, d, generator=g).bfloat16() for _ in range(3))
    do = torch.randn(1, s, heads, d, generator=g).bfloat16()
    orc.attention_ref(q[:, :256], k[:, :256], v[:, :256], causal=causal)   # warm-up

    def one():
        if not backward:
            orc.attention_ref(q, k, v, causal=causal)
            return
        qq, kk, vv = (x.clone().requires_grad_(True) for x in (q, k, v))
        out, _ = orc.attention_ref(qq, kk, vv, causal=causal)
        torch.autograd.grad(out, (qq, kk, vv), do)

    def run(budget):
        n, t0 = 0, time.perf_counter()
        while True:
            one()
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n >= 50:
                break
        fl = n * fwd_flops(1, heads, s, s, d, causal) * (3.5 if backward else 1.0)
        return fl, el, f"{n} x attention_ref{'+autograd bwd' if backward else ''}" \
                       f"(1x{s}x{heads}x{d} bf16->fp32, causal={causal})"

    if backward:
        qq, kk, vv = (x[:, :256].clone().requires_grad_(True) for x in (q, k, v))
        out, _ = orc.attention_ref(qq, kk, vv, causal=causal)      # autograd warm-up
        torch.autograd.grad(out, (qq, kk, vv), do[:, :256])
    med, rates, sample = _median_runs(run, reps, budget_s)
    return {"value": round(med / 1e12, 4), "unit": "TFLOP/s", "cores": threads, "kind": "port",
            "runs": [round(r / 1e12, 4) for r in rates], "cpu": _host(),
            "sample": f"median of {reps} runs of ~{budget_s / reps:.1f}s, last: {sample}"}


def cpu_baseline_decode(h: int, hk: int, s: int, d: int, budget_s: float, reps: int = 3):
    """Decode on the CPU oracle: one query token against an s-token cache (the fp8 cache
    dequantised to bf16, as the reference path would hold it), `reps` runs; reported as GB/s
    of the same algorithmic bytes the GPU line counts (fp8 K+V), median run."""
    from oracle import attention_ref as orc
    threads = _threads()
    g = torch.Generator().manual_seed(0)
    q = torch.randn(1, 1, h, d, generator=g).bfloat16()
    k, v = (torch.randn(1, s, hk, d, generator=g).bfloat16() for _ in range(2))
    orc.attention_ref(q, k[:, :256], v[:, :256])

    def run(budget):
        n, t0 = 0, time.perf_counter()
        while True:
            orc.attention_ref(q, k, v)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n >= 200:
                break
        nbytes = n * (2 * s * hk * d * 1 + 2 * h * d * 2)
        return nbytes, el, f"{n} x attention_ref(q 1x1x{h}x{d}, K/V 1x{s}x{hk}x{d} bf16->fp32)"

    med, rates, sample = _median_runs(run, reps, budget_s)
    return {"value": round(med / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "runs": [round(r / 1e9, 3) for r in rates], "cpu": _host(),
            "sample": f"median of {reps} runs of ~{budget_s / reps:.1f}s, last: {sample}"}


# ----------------------------------------------------------------------------- workloads
def varlen_lengths(n=32, total=131072, lo=1024, hi=7168, seed=0):
    """n lengths uniform in [lo, hi] from a seeded PRNG, rescaled so the sum
    is exactly `total` (the last one absorbs the rounding; with seed 0 the raw draw already
    sums past `total`, so adjusting only the last length would not do)."""
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(lo, hi + 1, (n,), generator=g).double()
    lens = (lens * total / lens.sum()).round().long()
    lens[-1] += total - int(lens.sum())
    return [int(x) for x in lens]


def _set_options(opts):
    from xf_flash_attention_cutlass_amd import capi
    for o in opts:                       # schedule knobs (fmha_set_option), A/B runs only
        name, val = o.split("=")
        if capi.lib().fmha_set_option(name.encode(), int(val)) != 0:
            raise SystemExit(capi.lib().fmha_last_error().decode())


def _rotating(sets):
    """Step closure helper: returns next() cycling through the input sets."""
    state = {"i": 0}

    def nxt():
        s = sets[state["i"] % len(sets)]
        state["i"] += 1
        return s
    return nxt


def workload_dense(a, mode, dev, rank, world):
    """C2 (mode fwd) / C3 (mode fwdbwd).  weak: B per rank; strong: this rank's head shard."""
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import sharding
    pa = xfa.paged_attn
    B, S, H, D = a.batch or 4, a.seqlen or 4096, a.heads, a.headdim
    causal = not a.no_causal
    scale = D ** -0.5
    Hr, shard = H, f"batch shard {B} of global {B * world}"
    if a.scaling == "strong":
        qs, _ = sharding.head_shards(H, H, world)[rank]
        Hr, shard = qs.size, f"heads [{qs.start}, {qs.stop}) of {H}"
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    nrot = a.rotate or 2
    sets = []
    for _ in range(nrot):
        q, k, v = (torch.randn(B, S, Hr, D, device=dev, dtype=torch.bfloat16, generator=g)
                   for _ in range(3))
        out = torch.empty_like(q)
        dout = torch.randn_like(q)
        sets.append((q, k, v, out, dout))
    nxt = _rotating(sets)
    res = {}
    wl = a.window_left
    alibi = (torch.tensor([2.0 ** (-8.0 * (i + 1) / H) for i in range(H)], device=dev)[:Hr]
             if a.alibi else None)

    def fwd():
        q, k, v, out, _ = nxt()
        res["r"] = pa.fwd(q, k, v, out, alibi, 0.0, scale, causal, wl, -1, 0.0, False, None)

    page = getattr(a, "page", 0) if mode == "fwd" else 0
    if page:
        # the same K / V laid into paged caches (one random-permutation block table per set)
        nbp = (S + page - 1) // page
        paged_sets = []
        for q, k, v, out, _ in sets:
            table = torch.randperm(B * nbp, device=dev, generator=g).int().view(B, nbp)
            kc = torch.zeros(B * nbp, page, Hr, D, device=dev, dtype=torch.bfloat16)
            vc = torch.zeros_like(kc)
            kc.view(-1, Hr, D)[(table.long().view(B, nbp, 1) * page +
                                torch.arange(page, device=dev)).view(B, -1)[:, :S].reshape(-1)] = k.reshape(-1, Hr, D)
            vc.view(-1, Hr, D)[(table.long().view(B, nbp, 1) * page +
                                torch.arange(page, device=dev)).view(B, -1)[:, :S].reshape(-1)] = v.reshape(-1, Hr, D)
            paged_sets.append((q, kc, vc, table))
        seqlens = torch.full((B,), S, dtype=torch.int32, device=dev)
        pnxt = _rotating(paged_sets)

        def fwd():      # noqa: F811
            q, kc, vc, table = pnxt()
            res["r"] = pa.fwd_kvcache(q, kc, vc, None, None, seqlens, None, None, None, table, alibi,
                                      None, scale, causal, wl, -1, 0.0, True, 1, None)

    def fwdbwd():
        q, k, v, out, dout = nxt()
        r = pa.fwd(q, k, v, out, alibi, 0.0, scale, causal, wl, -1, 0.0, False, None)
        pa.bwd(dout, q, k, v, out, r[5], None, None, None, alibi, 0.0, scale, causal, wl, -1,
               0.0, False, None, None)
        res["r"] = r

    ff = fwd_flops(B, Hr, S, S, D, causal)
    if wl >= 0:    # (sq = sk) row pos sees keys max(0, pos - wl) .. pos (causal) or .. pos + wl
        vis = sum(min(p, wl) + 1 + (0 if causal else min(S - 1 - p, wl)) for p in range(S))
        ff = 4.0 * B * Hr * D * vis
    mult = 3.5 if mode == "fwdbwd" else 1.0
    cs = ("causal" if causal else "non-causal") + (" ALiBi" if a.alibi else "") + \
        (f" window ({wl}, {0 if causal else wl})" if wl >= 0 else "") + \
        (f", paged K/V (page {page}, random block table)" if page else "")
    glob_b = B * world if a.scaling == "weak" else B
    return dict(step=fwd if mode == "fwd" else fwdbwd, units=ff * mult, bound="mfma",
                out=lambda: sets[0][3], gather_dim=0 if a.scaling == "weak" else 2,
                config={"workload": f"mha_{mode} B={B} H={H} S={S} D={D} bf16 {cs}",
                        "global_batch": glob_b, "seq_len": S, "heads": H, "head_dim": D,
                        "rank_shard": shard, "input_sets": nrot,
                        "parallelism": f"dp{world} ({a.scaling} scaling: "
                                       f"{'batch' if a.scaling == 'weak' else 'GQA-aligned head'}"
                                       f" shards, no collective in the step)"},
                cpu=lambda: cpu_baseline_dense(8 if mode == "fwd" else 2, S, D, causal,
                                               a.cpu_baseline_seconds, backward=mode == "fwdbwd"))


def workload_fp8(a, dev, rank, world):
    """C2 shape with fp8 e4m3fn Q/K/V (per-tensor descales), bf16 output."""
    import xf_flash_attention_cutlass_amd as xfa
    pa = xfa.paged_attn
    B, S, H, D = a.batch or 4, a.seqlen or 4096, a.heads, a.headdim
    causal = not a.no_causal
    scale = D ** -0.5
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    sets = []
    for _ in range(a.rotate or 2):
        xs = []
        for _ in range(3):
            t = torch.randn(B, S, H, D, device=dev, generator=g)
            s8 = float(t.abs().max()) / 448.0
            xs.append(((t / s8).to(torch.float8_e4m3fn), s8))
            del t
        out = torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16)
        sets.append((xs, out))
    nxt = _rotating(sets)

    def step():
        (q, qs), (k, ks), (v, vs) = (x for x in nxt()[0])
        pa.fwd_fp8(q, k, v, None, qs, ks, vs, scale, causal, -1, -1, False)

    cs = "causal" if causal else "non-causal"
    return dict(step=step, units=fwd_flops(B, H, S, S, D, causal), bound="mfma8",
                out=lambda: sets[0][1], gather_dim=0,
                config={"workload": f"mha_fwd fp8-e4m3 Q/K/V B={B} H={H} S={S} D={D} {cs}, "
                                    f"bf16 out", "global_batch": B * world, "seq_len": S,
                        "heads": H, "head_dim": D, "input_sets": a.rotate or 2,
                        "parallelism": f"dp{world} ({a.scaling} scaling: batch shards)"},
                cpu=lambda: cpu_baseline_dense(8, S, D, causal, a.cpu_baseline_seconds))


def workload_varlen(a, dev, rank, world):
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import sharding
    pa = xfa.paged_attn
    H, D = a.heads, a.headdim
    causal = not a.no_causal
    scale = D ** -0.5
    if a.scaling == "weak":
        lens = varlen_lengths(seed=rank)        # every rank its own 32 sequences
        shard = f"32 sequences of global {32 * world}"
    else:
        all_lens = varlen_lengths()
        mine = sharding.balanced_sequences(all_lens, all_lens, world)[rank]
        lens = [all_lens[i] for i in mine]
        shard = f"sequences {mine}"
    tot = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=dev)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    q, k, v = (torch.randn(tot, H, D, device=dev, dtype=torch.bfloat16, generator=g)
               for _ in range(3))
    out = torch.empty_like(q)
    mx = max(lens)

    def step():
        pa.varlen_fwd(q, k, v, out, cu, cu, None, None, None, mx, mx, 0.0, scale, False,
                      causal, -1, -1, 0.0, False, None)

    fl = sum(fwd_flops(1, H, s, s, D, causal) for s in lens)
    cs = "causal" if causal else "non-causal"
    return dict(step=step, units=fl, bound="mfma", out=lambda: out, gather_dim=0,
                config={"workload": f"mha_varlen_fwd 32 ragged seqs, lengths {min(lens)}-{max(lens)} "
                                    f"(U[1024,7168] draw, seed {rank}, rescaled to total 131072) "
                                    f"H={H} D={D} bf16 {cs}",
                        "global_batch": 32 * world if a.scaling == "weak" else 32,
                        "seq_len": mx, "total_tokens": tot, "heads": H, "head_dim": D,
                        "rank_shard": shard,
                        "parallelism": f"dp{world} ({a.scaling} scaling: sequence shards, "
                                       f"no collective)"},
                cpu=lambda: cpu_baseline_dense(8, lens[0], D, causal, a.cpu_baseline_seconds))


def workload_decode(a, dev, rank, world):
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import sharding
    pa = xfa.paged_attn
    H, D, HK, page = a.heads, a.headdim, 8, 16
    S = a.seqlen or 32768
    scale = D ** -0.5
    if a.scaling == "weak":
        B = a.batch or 8
        shard = f"batch {B} of global {B * world}"
        glob_b = B * world
    else:
        glob_b = a.batch or 64
        bs = sharding.batch_shards(glob_b, world)[rank]
        B = bs.size
        shard = f"batch rows [{bs.start}, {bs.stop}) of {glob_b}"
    nblk_seq = S // page
    nblocks = B * nblk_seq
    if a.ragged:
        gl = torch.Generator().manual_seed(rank)
        lens = torch.randint(1, S + 1, (B,), generator=gl).to(torch.int32)
    else:
        lens = torch.full((B,), S, dtype=torch.int32)
    seqlens = lens.to(dev)
    gp = torch.Generator().manual_seed(rank)
    table = torch.randperm(nblocks, generator=gp).to(torch.int32).view(B, nblk_seq).to(dev)
    ks, vs = 1.0 / 16, 1.0 / 16
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    kc = torch.empty(nblocks, page, HK, D, device=dev, dtype=torch.uint8)
    vc = torch.empty_like(kc)
    for c, sc_ in ((kc, ks), (vc, vs)):      # chunked to bound the bf16 temporary
        for i in range(0, nblocks, 4096):
            t = torch.randn(min(4096, nblocks - i), page, HK, D, device=dev,
                            dtype=torch.bfloat16, generator=g)
            c[i:i + t.shape[0]] = (t.float() / sc_).to(torch.float8_e4m3fn).view(torch.uint8)
    q = torch.randn(B, 1, H, D, device=dev, dtype=torch.bfloat16, generator=g)
    res = {}

    def step():
        res["o"] = pa.fwd_kvcache_fp8(q, kc, vc, seqlens, table, ks, vs, scale, False, -1, -1,
                                      0)[0]

    step()
    nbytes = int(lens.sum()) * HK * D * 2 + 2 * B * H * D * 2 + table.numel() * 4 + B * 4
    return dict(step=step, units=nbytes, bound="hbm", out=lambda: res["o"], gather_dim=0,
                config={"workload": f"paged-KV decode B={B}/GPU H={H} Hk={HK} Sq=1 "
                                    f"cache={'U[1,%d]' % S if a.ragged else S} page={page} "
                                    f"D={D} fp8-e4m3fn K/V (scale 1/16), q bf16",
                        "global_batch": glob_b, "seq_len": S, "heads": H, "head_dim": D,
                        "rank_shard": shard,
                        "parallelism": f"dp{world} ({a.scaling} scaling: batch shards, each "
                                       f"rank owns its sequences' pages, no collective)"},
                cpu=lambda: cpu_baseline_decode(H, HK, S, D, min(a.cpu_baseline_seconds, 10)))


def build_workload(a, mode, dev, rank, world):
    if mode in ("fwd", "fwdbwd"):
        return workload_dense(a, mode, dev, rank, world)
    if mode == "varlen":
        return workload_varlen(a, dev, rank, world)
    if mode == "fwd_fp8":
        return workload_fp8(a, dev, rank, world)
    return workload_decode(a, dev, rank, world)


def measured_traffic(mode):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary
    (profiles/r*_traffic.json, written by tools/pmc_report.py from rocprofv3 --pmc passes with
    the gfx950 FETCH_SIZE x2 correction), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return None
    for f in reversed(files):            # the newest summary that profiled this mode
        try:
            d = json.load(open(f)).get(mode)
        except (OSError, ValueError):
            continue
        if d is not None and "hbm_bytes_per_launch" in d:
            return {"bytes": d["hbm_bytes_per_launch"], "file": os.path.relpath(f, ROOT)}
    return None


def event_ms(step, steps, stream):
    """Per-step times from HIP events recorded on the launch stream around every step (a
    separate pass: the event records do not sit in the wall-clock timed region): (median, min,
    max) in ms."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    for i in range(steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in evs)
    return ts[len(ts) // 2], ts[0], ts[-1]


class ClockMonitor:
    """tools/gpu_monitor.py as a child process started BEFORE this process touches the GPU (it
    samples `amd-smi metric` clocks and socket power about every 0.1 s; nothing is exec'd from a
    process that has initialised the GPU).  stats(t0, t1) summarises the samples in a window."""

    def __init__(self):
        import tempfile
        self.path = os.path.join(tempfile.mkdtemp(prefix="xfa_mon_"), "samples.jsonl")
        self.proc = None
        try:
            self.proc = subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "tools", "gpu_monitor.py"), self.path],
                stdin=subprocess.PIPE, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except OSError:
            self.proc = None

    def select(self, pci_bus):
        """Point the sampler at this process' device (amd-smi numbers all of the machine's
        GPUs, whatever HIP_VISIBLE_DEVICES says)."""
        self.bdf = pci_bus.lower()
        if self.proc:
            try:
                self.proc.stdin.write(f"bdf {self.bdf}\n".encode())
                self.proc.stdin.flush()
            except OSError:
                pass

    def samples(self):
        try:
            with open(self.path) as f:
                return [json.loads(x) for x in f if x.strip()]
        except (OSError, ValueError):
            return []

    def stats(self, t0, t1):
        ss = [x for x in self.samples() if t0 <= x["t"] <= t1 and x.get("gfx_mhz")]
        want = getattr(self, "bdf", None)
        mine = [x for x in ss if want and str(x.get("bdf") or "").startswith(want)]
        # samples of this process' own GPU when amd-smi matched its BDF; otherwise amd-smi's
        # GPU 0, flagged as possibly another GPU of the machine
        matched = bool(mine)
        ss = mine or ss
        if not ss:
            return {"samples": 0, "source": "amd-smi metric (no samples in the window)"}
        per = sorted(sum(x["gfx_mhz"]) / len(x["gfx_mhz"]) for x in ss)   # mean over XCDs
        pw = sorted(x["power_w"] for x in ss if isinstance(x.get("power_w"), (int, float)))
        med = lambda v: v[len(v) // 2] if v else None   # noqa: E731
        return {"samples": len(ss), "window_s": round(t1 - t0, 3),
                "gfx_mhz_median": round(med(per), 1), "gfx_mhz_min": round(per[0], 1),
                "gfx_mhz_max": round(per[-1], 1),
                "power_w_median": med(pw), "power_w_max": pw[-1] if pw else None,
                "bdf": ss[-1].get("bdf"), "bdf_match": matched,
                "source": "amd-smi metric -c -p (current gfx clock, mean over XCDs; socket power)"}

    def close(self):
        if self.proc:
            try:
                self.proc.stdin.close()
                self.proc.wait(timeout=5)
            except (OSError, subprocess.SubprocessError):
                self.proc.kill()
            self.proc = None
        import shutil
        shutil.rmtree(os.path.dirname(self.path), ignore_errors=True)


MONITOR = None


def clock_stats(t0, t1):
    return MONITOR.stats(t0, t1) if MONITOR else None


def device_info(dev):
    pr = torch.cuda.get_device_properties(dev)
    return {"name": pr.name, "arch": pr.gcnArchName, "cus": pr.multi_processor_count,
            "pci_bus": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
            "hbm_gib": round(pr.total_memory / 2 ** 30, 1)}


def last_kernel():
    from xf_flash_attention_cutlass_amd import capi
    return capi.lib().fmha_last_kernel().decode() or None


def prewarm(step, seconds, sync):
    """GPU clock ramp: an idle MI355X needs a few hundred ms of sustained load to reach its
    steady clock (measured: 20 steps after 5 warmups read 12 % low on C2)."""
    t = time.perf_counter()
    while time.perf_counter() - t < seconds:
        for _ in range(8):
            step()
        sync()


def traffic_key(a, mode):
    """the tools/pmc_round.sh mode whose measured HBM bytes belong to this run's kernel"""
    if mode == "decode":
        return "decode_ragged" if a.ragged else "decode"
    if mode == "fwd":
        if getattr(a, "alibi", False):
            return "fwd_alibi"
        if getattr(a, "window_left", -1) >= 0:
            return "fwd_window"
        if getattr(a, "page", 0):
            return "fwd_paged"
        if a.no_causal:
            return "fwd_nc"
    return mode


def roofline(w, ev, mode):
    ms, ms_min, ms_max = ev
    hbm = w["bound"] == "hbm"
    scale_u = 1e9 if hbm else 1e12
    achieved = w["units"] / (ms / 1e3) / scale_u
    peak = PEAK_HBM_GBS if hbm else PEAK_FP8_TFLOPS if w["bound"] == "mfma8" else PEAK_BF16_TFLOPS
    tr = measured_traffic(mode)
    roof = {"bound": "mfma" if w["bound"] == "mfma8" else w["bound"], "achieved": round(achieved, 2), "peak": peak,
            "unit": "GB/s" if hbm else "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": tr["bytes"] if tr else None,
            "algorithmic_per_launch": w["units"], "kernel_ms": round(ms, 4),
            "kernel_ms_min": round(ms_min, 4), "kernel_ms_max": round(ms_max, 4)}
    if tr:
        roof["traffic_source"] = tr["file"]
    return roof


def sub_result(a, mode, dev, stream, **over):
    """A driver-timed sub-result (same method as the main line, rank-local, 1 GPU), with its
    own CPU baseline; `over` overrides arguments (e.g. ragged=True)."""
    a = argparse.Namespace(**{**vars(a), **over})
    w = build_workload(a, mode, dev, 0, 1)
    step = w["step"]
    t_pw = time.time()
    prewarm(step, 0.5, torch.cuda.synchronize)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    k = max(10, a.steps)
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) / k * 1e3
    ev = event_ms(step, k, stream)
    t_end = time.time()
    hbm = w["bound"] == "hbm"
    u = 1e9 if hbm else 1e12
    out = {"workload": w["config"]["workload"], "steps": k, "ms_per_step": round(wall_ms, 4),
           "value": round(w["units"] / (wall_ms / 1e3) / u, 2),
           "unit": "GB/s" if hbm else "TFLOP/s",
           "roofline": roofline(w, ev, getattr(a, "roof_key", None) or traffic_key(a, mode)),
           "kernel": last_kernel(),
           "gpu_clock": clock_stats(t_pw + 0.2, t_end)}
    if not a.no_cpu_baseline:
        out["cpu_baseline"] = w["cpu"]()
    del w
    torch.cuda.empty_cache()
    return out


# ----------------------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a, argv):
    """Start N ranks as a child `torch.distributed.run` on this file (this process has not
    touched the GPU and never execs: it waits for the child and returns its status)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def selftest_cpu(a, rank, world):
    """Launcher / barrier / max-over-ranks self-test on CPU with gloo (not a benchmark)."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    x = torch.randn(256, 256)
    step = lambda: x @ x          # noqa: E731
    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        units = 2.0 * 256 ** 3 * a.steps * world
        print(json.dumps({"metric": "bench launcher self-test (CPU gloo; not a benchmark)",
                          "value": round(units / t.item() / 1e9, 3), "unit": "GFLOP/s",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(t.item() / a.steps * 1e3, 4),
                          "world_size": world,
                          "backend": dist.get_backend() if world > 1 else None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch with "
                         f"--nproc-per-node {a.gpus} (or let bench.py launch the ranks)")
    a.world = world
    if a.selftest_cpu:
        return selftest_cpu(a, rank, world)

    global MONITOR
    # under a profiler (rocprofv3's preloaded library initialises the GPU before this program
    # starts) no child process is started at all
    profiled = any(k.startswith("ROCPROF") for k in os.environ) or \
        "rocprof" in os.environ.get("LD_PRELOAD", "")
    if world == 1 and not a.no_monitor and not profiled:
        MONITOR = ClockMonitor()         # before this process touches the GPU
    try:
        return run(a, world, rank, local)
    finally:
        if MONITOR:
            MONITOR.close()


def run(a, world, rank, local):
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if MONITOR:
        MONITOR.select(device_info(dev)["pci_bus"])   # sample this rank's own GPU
    dist = None
    if world > 1 or "WORLD_SIZE" in os.environ:
        # (a one-rank group too when launched by torch.distributed.run: the sharded path runs
        # as at N > 1, but at world size 1 no collective is issued — all_gather_dim returns the
        # local shard — so the all-gather line then times nothing)
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    _set_options(a.opt)

    w = build_workload(a, a.mode, dev, rank, world)
    step = w["step"]
    # Optional: replay a captured hipGraph of one step (same kernels).  Measured on C5 decode
    # it is slower than eager launches on this stack (0.136 vs 0.129 ms per step), so eager
    # is the default.
    use_graph = a.graph == "on"
    if use_graph:
        gs = torch.cuda.Stream()
        with torch.cuda.stream(gs):          # per-stream scratch is allocated before capture
            for _ in range(2):
                step()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=gs):
            step()
        torch.cuda.synchronize()
        step = graph.replay
    t_pw = time.time()
    prewarm(step, a.prewarm_s, torch.cuda.synchronize)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # kernels launch on torch's current stream; HIP events go on that stream
    stream = torch.cuda.current_stream()

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):              # the timed region: exactly K steps, nothing else
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ev_ms = event_ms(step, a.steps, stream)
    t_end = time.time()
    kern = last_kernel()

    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    units = torch.tensor([w["units"]], device=dev, dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(units, op=dist.ReduceOp.SUM)
    elapsed, total_units = t.item(), units.item()

    hbm = w["bound"] == "hbm"
    scale_u = 1e9 if hbm else 1e12
    value = total_units * a.steps / elapsed / scale_u
    ms_per_step = elapsed / a.steps * 1e3

    allgather = None
    if dist:
        out = w["out"]()
        gd = w["gather_dim"]
        # RCCL all-gather of every rank's output shard over xGMI (assembling the full output)
        from xf_flash_attention_cutlass_amd import sharding
        n_local = torch.tensor([out.shape[gd]], device=dev)
        sizes = [torch.zeros_like(n_local) for _ in range(world)]
        dist.all_gather(sizes, n_local)
        sizes = [int(s.item()) for s in sizes]
        for _ in range(3):
            sharding.all_gather_dim(out, sizes, gd)
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(10):
            full = sharding.all_gather_dim(out, sizes, gd)
        torch.cuda.synchronize()
        ag = torch.tensor([(time.perf_counter() - t1) / 10], device=dev, dtype=torch.float64)
        dist.all_reduce(ag, op=dist.ReduceOp.MAX)
        ag_ms = ag.item() * 1e3
        allgather = {"ms": round(ag_ms, 3), "gathered_shape": list(full.shape),
                     "bytes_per_rank_in": out.numel() * out.element_size() * (world - 1),
                     "value_with_gather": round(total_units / ((ms_per_step + ag_ms) / 1e3)
                                                / scale_u, 2)}

    extras = {}
    if rank == 0 and a.mode == "fwd" and world == 1 and not a.no_extras:
        extras["fwd_bwd"] = sub_result(a, "fwdbwd", dev, stream)
        extras["varlen"] = sub_result(a, "varlen", dev, stream)
        extras["decode"] = sub_result(a, "decode", dev, stream)
        extras["decode_ragged"] = sub_result(a, "decode", dev, stream, ragged=True)
        extras["fwd_fp8"] = sub_result(a, "fwd_fp8", dev, stream)
        # north_star's target shape names no mask: the same C2 shape non-causal; and the C2 shape
        # with the two masks the reference's kernel also takes, causal ALiBi and a causal
        # 1024-key sliding window (no CPU baselines for these three)
        extras["fwd_noncausal"] = sub_result(a, "fwd", dev, stream, no_causal=True,
                                             no_cpu_baseline=True, roof_key="fwd_nc")
        extras["fwd_alibi"] = sub_result(a, "fwd", dev, stream, alibi=True, no_cpu_baseline=True,
                                         roof_key="fwd_alibi")
        extras["fwd_paged"] = sub_result(a, "fwd", dev, stream, page=16, no_cpu_baseline=True,
                                         roof_key="fwd_paged")
        extras["fwd_window"] = sub_result(a, "fwd", dev, stream, window_left=1023,
                                          no_cpu_baseline=True, roof_key="fwd_window")
    if dist:
        dist.barrier()

    if rank == 0:
        from xf_flash_attention_cutlass_amd import capi
        line = {
            "metric": METRIC if not hbm else "paged-KV decode HBM GB/s (C5)",
            "value": round(value, 2),
            "unit": "GB/s" if hbm else "TFLOP/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": ("fp8-e4m3 K/V, bf16 q/o, f32 accumulate" if hbm else
                      "fp8-e4m3 q/k/v and P, bf16 out, f32 accumulate" if a.mode == "fwd_fp8"
                      else "bf16"),
            "data": "synthetic (torch.randn, N(0,1)), inputs resident in HBM",
            "prewarm_s": a.prewarm_s,
            "launch": "hipGraph replay of one step" if use_graph else "eager",
            "options": dict(o.split("=") for o in a.opt),
            "library": capi.lib().fmha_version().decode(),
            "config": w["config"],
            "roofline": roofline(w, ev_ms, a.mode + ("_ragged" if a.ragged else "")),
            "kernel": kern,
            "device": device_info(dev),
            "gpu_clock": clock_stats(t_pw + 0.2, t_end),
        }
        if dist:
            line["rccl"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
        line.update(extras)
        if allgather:
            line["allgather"] = allgather
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = w["cpu"]()
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

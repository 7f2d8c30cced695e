"""Benchmark of the hot path on MI355X (BASELINE.json metric: attention TFLOPS/GPU).

Workloads (BASELINE.json configs):
  --mode fwd     (default) C2: mha_fwd B=4 H=32 S=4096 D=128 bf16 causal; one step = one
                 forward over the batch.  The line also carries a short C3 (fwd+bwd) sample
                 under "fwd_bwd" because the metric names both.
  --mode fwdbwd  C3: mha_fwd + mha_bwd, same shape (FLOPs = 3.5 x fwd, the usual convention).
  --mode varlen  C4: mha_varlen_fwd, 32 ragged sequences, total 131072 tokens, H=32 D=128 bf16.
  --mode decode  C5: paged-KV decode (fwd_kvcache), per GPU B=8 H=32 Hk=8 Sq=1, cache 32768
                 tokens, page 16, fp8 e4m3fn K/V; HBM-bound, reported in GB/s.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode fwd|fwdbwd|varlen|decode]

N > 1 is launched by torch.distributed.run (one process per GPU): every rank owns its own
shard of independent (batch, head) / sequence units — attention has no cross-unit reduction,
so the timed region has no collective ("scaling": "weak"); the RCCL all-gather of outputs
over xGMI that assembles the sharded result is timed separately under "allgather".

Prints ONE JSON line on rank 0 (value = whole-job throughput summed over all ranks).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md §HBM)
METRIC = "attention TFLOPS/GPU (fwd, fwd+bwd) at S=4096 D=128; % MI355X MFMA peak"


def fwd_flops(b, h, sq, sk, d, causal):
    f = 4.0 * b * h * sq * sk * d
    return f / 2 if causal else f


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["fwd", "fwdbwd", "varlen", "decode"], default="fwd")
    ap.add_argument("--batch", type=int, default=0, help="default: 4 (fwd), 8 (decode)")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--seqlen", type=int, default=0, help="default: 4096 (fwd), 32768 (decode)")
    ap.add_argument("--headdim", type=int, default=128)
    ap.add_argument("--no-causal", action="store_true")
    ap.add_argument("--ragged", action="store_true", help="decode: cache lengths U[1, S]")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the fwd_bwd sample")
    ap.add_argument("--graph", choices=["on", "off"], default="off",
                    help="replay one step as a captured hipGraph")
    ap.add_argument("--opt", action="append", default=[],
                    help="name=value tuning option (fmha_set_option) for A/B runs")
    ap.add_argument("--prewarm-s", type=float, default=1.0,
                    help="untimed seconds of steps before the warmup (GPU clock ramp)")
    return ap.parse_args()


# ----------------------------------------------------------------------------- CPU baselines
def _threads():
    t = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    torch.set_num_threads(t)
    return t


def _host():
    return platform.processor() or platform.machine()


def cpu_baseline_dense(heads: int, s: int, d: int, causal: bool, budget_s: float):
    """Reference CPU eager path (oracle restatement of test.py:310-397, fp32 upcast) timed on
    the host cores over a bounded sample: repeated (1 batch x `heads` heads) chunks of the
    same workload until `budget_s` seconds of work; reported in TFLOP/s."""
    from oracle import attention_ref as orc
    threads = _threads()
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(1, s, heads, d, generator=g).bfloat16() for _ in range(3))
    orc.attention_ref(q[:, :256], k[:, :256], v[:, :256], causal=causal)   # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        orc.attention_ref(q, k, v, causal=causal)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 50:
            break
    flops = n * fwd_flops(1, heads, s, s, d, causal)
    return {"value": round(flops / el / 1e12, 4), "unit": "TFLOP/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} x attention_ref(1x{s}x{heads}x{d} bf16->fp32, causal={causal}) "
                      f"in {el:.1f}s on {_host()}"}


def cpu_baseline_decode(h: int, hk: int, s: int, d: int, budget_s: float):
    """Decode on the CPU oracle: one query token against an s-token cache (the fp8 cache
    dequantised to bf16, as the reference path would hold it), repeated for `budget_s`;
    reported as GB/s of the same algorithmic bytes the GPU line counts (fp8 K+V)."""
    from oracle import attention_ref as orc
    threads = _threads()
    g = torch.Generator().manual_seed(0)
    q = torch.randn(1, 1, h, d, generator=g).bfloat16()
    k, v = (torch.randn(1, s, hk, d, generator=g).bfloat16() for _ in range(2))
    orc.attention_ref(q, k[:, :256], v[:, :256])
    n, t0 = 0, time.perf_counter()
    while True:
        orc.attention_ref(q, k, v)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 200:
            break
    nbytes = n * (2 * s * hk * d * 1 + 2 * h * d * 2)
    return {"value": round(nbytes / el / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} x attention_ref(q 1x1x{h}x{d}, K/V 1x{s}x{hk}x{d} bf16->fp32) "
                      f"in {el:.1f}s on {_host()}"}


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


def build_workload(a, dev, rank):
    """Returns dict(step, units, bound, config, cpu, out) for the selected mode; `units` is
    the algorithmic FLOPs (mfma-bound) or bytes (hbm-bound) one step processes."""
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    for o in a.opt:                       # tuning knobs (fmha_set_option), A/B runs only
        name, val = o.split("=")
        if capi.lib().fmha_set_option(name.encode(), int(val)) != 0:
            raise SystemExit(capi.lib().fmha_last_error().decode())
    pa = xfa.paged_attn
    H, D = a.heads, a.headdim
    causal = not a.no_causal
    scale = D ** -0.5
    g = torch.Generator(device=dev).manual_seed(1234 + rank)   # each rank: its own shard
    cs = "causal" if causal else "non-causal"

    if a.mode in ("fwd", "fwdbwd"):
        B, S = a.batch or 4, a.seqlen or 4096
        q, k, v = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
                   for _ in range(3))
        out = torch.empty_like(q)
        dout = torch.randn_like(q)
        lse = pa.fwd(q, k, v, out, None, 0.0, scale, causal, -1, -1, 0.0, False, None)[5]

        def fwd():
            pa.fwd(q, k, v, out, None, 0.0, scale, causal, -1, -1, 0.0, False, None)

        def fwdbwd():
            r = pa.fwd(q, k, v, out, None, 0.0, scale, causal, -1, -1, 0.0, False, None)
            pa.bwd(dout, q, k, v, out, r[5], None, None, None, None, 0.0, scale, causal, -1, -1,
                   0.0, False, None, None)

        ff = fwd_flops(B, H, S, S, D, causal)
        mult = 3.5 if a.mode == "fwdbwd" else 1.0
        return dict(step=fwd if a.mode == "fwd" else fwdbwd, units=ff * mult, bound="mfma",
                    out=out, extra=(fwdbwd, ff * 3.5) if a.mode == "fwd" else None,
                    config={"workload": f"mha_{a.mode} B={B} H={H} S={S} D={D} bf16 {cs}",
                            "global_batch": B * a.world, "seq_len": S, "heads": H,
                            "head_dim": D,
                            "parallelism": f"dp{a.world} (batch x head shards, no collective "
                                           f"in step)"},
                    cpu=lambda: cpu_baseline_dense(8, S, D, causal, a.cpu_baseline_seconds))

    if a.mode == "varlen":
        lens = varlen_lengths()
        tot = sum(lens)
        cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32,
                          device=dev)
        q, k, v = (torch.randn(tot, H, D, device=dev, dtype=torch.bfloat16, generator=g)
                   for _ in range(3))
        out = torch.empty_like(q)
        mx = max(lens)

        def step():
            pa.varlen_fwd(q, k, v, out, cu, cu, None, None, None, mx, mx, 0.0, scale, False,
                          causal, -1, -1, 0.0, False, None)

        fl = sum(fwd_flops(1, H, s, s, D, causal) for s in lens)
        s0 = lens[0]
        return dict(step=step, units=fl, bound="mfma", out=out, extra=None,
                    config={"workload": f"mha_varlen_fwd {len(lens)} ragged seqs "
                                        f"U[1024,7168] (seed 0) total={tot} H={H} D={D} bf16 "
                                        f"{cs}", "global_batch": len(lens) * a.world,
                            "seq_len": mx, "total_tokens": tot, "heads": H, "head_dim": D,
                            "parallelism": f"dp{a.world} (sequence shards, no collective)"},
                    cpu=lambda: cpu_baseline_dense(8, s0, D, causal, a.cpu_baseline_seconds))

    # decode (C5)
    B, S, HK, page = a.batch or 8, a.seqlen or 32768, 8, 16
    nblk_seq = S // page
    nblocks = B * nblk_seq
    if a.ragged:
        gl = torch.Generator().manual_seed(rank)
        lens = torch.randint(1, S + 1, (B,), generator=gl).to(torch.int32)
    else:
        lens = torch.full((B,), S, dtype=torch.int32)
    seqlens = lens.to(dev)
    gp = torch.Generator().manual_seed(0)
    table = torch.randperm(nblocks, generator=gp).to(torch.int32).view(B, nblk_seq).to(dev)
    ks, vs = 1.0 / 16, 1.0 / 16
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
    return dict(step=step, units=nbytes, bound="hbm", out=res["o"], extra=None,
                config={"workload": f"paged-KV decode B={B} H={H} Hk={HK} Sq=1 "
                                    f"cache={'U[1,%d]' % S if a.ragged else S} page={page} "
                                    f"D={D} fp8-e4m3fn K/V (scale 1/16), q bf16",
                        "global_batch": B * a.world, "seq_len": S, "heads": H, "head_dim": D,
                        "parallelism": f"dp{a.world} (batch shards: each rank owns its "
                                       f"sequences' pages, no collective)"},
                cpu=lambda: cpu_baseline_decode(H, HK, S, D, min(a.cpu_baseline_seconds, 10)))


def measured_traffic(mode):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary
    (profiles/r*_traffic.json, written by tools/traffic.py from rocprofv3 --pmc passes with
    the gfx950 FETCH_SIZE x2 correction), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1])).get(mode)
        return None if d is None else {"bytes": d["hbm_bytes_per_launch"], "file":
                                       os.path.relpath(files[-1], ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def timed(step, steps, stream):
    """Run `steps` steps with HIP events on the launch stream; returns mean event ms."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    for i in range(steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    return sum(s.elapsed_time(e) for s, e in evs) / steps


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    a.world = world
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    w = build_workload(a, dev, rank)
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
    # GPU clock ramp: an idle MI355X needs a few hundred ms of sustained load to reach its
    # steady clock (measured: 20 steps after 5 warmups read 12 % low on C2).  Run the step
    # untimed for --prewarm-s seconds before the W warmup steps; the timed region is still
    # exactly K steps.
    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < a.prewarm_s:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # Kernel-level timing with HIP events on the stream the kernels are launched on
    # (paged_attn launches on torch's current stream).
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
    # kernel-level time per step (roofline "achieved"): a separate pass of K steps bracketed
    # by HIP events on the launch stream, so the event records do not sit in the timed region
    ev_ms = timed(step, a.steps, stream)

    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()

    hbm = w["bound"] == "hbm"
    scale_u = 1e9 if hbm else 1e12
    value = w["units"] * a.steps * world / elapsed / scale_u
    ms_per_step = elapsed / a.steps * 1e3

    allgather = None
    if dist:
        out = w["out"]
        # RCCL all-gather of every rank's O shard over xGMI (assembling the sharded output).
        gathered = torch.empty((world * out.shape[0],) + tuple(out.shape[1:]), device=dev,
                               dtype=out.dtype)
        for _ in range(3):
            dist.all_gather_into_tensor(gathered, out)
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(10):
            dist.all_gather_into_tensor(gathered, out)
        torch.cuda.synchronize()
        ag = torch.tensor([(time.perf_counter() - t1) / 10], device=dev, dtype=torch.float64)
        dist.all_reduce(ag, op=dist.ReduceOp.MAX)
        ag_ms = ag.item() * 1e3
        allgather = {"ms": round(ag_ms, 3),
                     "bytes_per_rank_in": out.numel() * out.element_size() * (world - 1),
                     "value_with_gather": round(w["units"] * world /
                                                ((ms_per_step + ag_ms) / 1e3) / scale_u, 2)}

    extra = None
    if w["extra"] and not a.no_extras:
        fn, units = w["extra"]
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ms = timed(fn, max(10, a.steps // 2), stream)
        extra = {"workload": "mha_fwd + mha_bwd (C3), same shape; FLOPs = 3.5 x fwd",
                 "ms_per_step": round(ms, 4), "tflops": round(units / (ms / 1e3) / 1e12, 2),
                 "frac": round(units / (ms / 1e3) / 1e12 / PEAK_BF16_TFLOPS, 4)}

    if rank == 0:
        achieved = w["units"] / (ev_ms / 1e3) / scale_u
        peak = PEAK_HBM_GBS if hbm else PEAK_BF16_TFLOPS
        tr = measured_traffic(a.mode)
        roof = {"bound": w["bound"], "achieved": round(achieved, 2), "peak": peak,
                "unit": "GB/s" if hbm else "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": tr["bytes"] if tr else None,
                "algorithmic_per_launch": w["units"], "kernel_ms": round(ev_ms, 4)}
        if tr:
            roof["traffic_source"] = tr["file"]
        line = {
            "metric": METRIC if not hbm else "paged-KV decode HBM GB/s (C5)",
            "value": round(value, 2),
            "unit": "GB/s" if hbm else "TFLOP/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if not hbm else "fp8-e4m3 K/V, bf16 q/o, f32 accumulate",
            "data": "synthetic (torch.randn, N(0,1)), inputs resident in HBM",
            "prewarm_s": a.prewarm_s,
            "launch": "hipGraph replay of one step" if use_graph else "eager",
            "config": w["config"],
            "roofline": roof,
        }
        if extra:
            line["fwd_bwd"] = extra
        if allgather:
            line["allgather"] = allgather
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = w["cpu"]()
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

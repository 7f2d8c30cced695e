"""Benchmark of the hot path on MI355X (BASELINE.json metric: attention TFLOPS/GPU).

Default workload = BASELINE.json configs[1]: mha_fwd B=4 H=32 S=4096 D=128 bf16 causal,
one step = one forward over the batch.  `--mode fwdbwd` times configs[2] (fwd + bwd).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode fwd|fwdbwd]

N > 1 is launched by torch.distributed.run (one process per GPU): every rank owns its own
B x H shard of (batch, head) units — attention has no cross-unit reduction in fwd, so the
timed region has no collective ("scaling": "weak"); the RCCL all-gather of outputs over xGMI
that assembles the sharded result is timed separately and reported under "allgather".

Prints ONE JSON line on rank 0 (value = whole-job TFLOP/s summed over all ranks).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def fwd_flops(b, h, sq, sk, d, causal):
    f = 4.0 * b * h * sq * sk * d
    return f / 2 if causal else f


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["fwd", "fwdbwd"], default="fwd")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--seqlen", type=int, default=4096)
    ap.add_argument("--headdim", type=int, default=128)
    ap.add_argument("--no-causal", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(b_heads: int, s: int, d: int, causal: bool, budget_s: float):
    """Reference CPU eager path (oracle restatement of test.py:310-397, fp32 upcast) timed on
    the host cores over a bounded sample: repeated (1 batch x `b_heads` heads) chunks of the
    same workload until `budget_s` seconds of work; reported in the same TFLOP/s unit."""
    from oracle import attention_ref as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    q = torch.randn(1, s, b_heads, d, generator=g).bfloat16()
    k = torch.randn(1, s, b_heads, d, generator=g).bfloat16()
    v = torch.randn(1, s, b_heads, d, generator=g).bfloat16()
    orc.attention_ref(q[:, :256], k[:, :256], v[:, :256], causal=causal)   # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        orc.attention_ref(q, k, v, causal=causal)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 50:
            break
    flops = n * fwd_flops(1, b_heads, s, s, d, causal)
    return {"value": round(flops / el / 1e12, 4), "unit": "TFLOP/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} x attention_ref(1x{s}x{b_heads}x{d} bf16->fp32, causal={causal}) "
                      f"in {el:.1f}s on {platform.processor() or platform.machine()}"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import xf_flash_attention_cutlass_amd as xfa
    pa = xfa.paged_attn
    B, H, S, D = a.batch, a.heads, a.seqlen, a.headdim
    causal = not a.no_causal
    scale = D ** -0.5
    g = torch.Generator(device=dev).manual_seed(1234 + rank)   # each rank: its own shard
    q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
    k = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
    out = torch.empty_like(q)
    dout = torch.randn_like(q) if a.mode == "fwdbwd" else None

    def step():
        r = pa.fwd(q, k, v, out, None, 0.0, scale, causal, -1, -1, 0.0, False, None)
        if a.mode == "fwdbwd":
            pa.bwd(dout, q, k, v, out, r[5], None, None, None, None, 0.0, scale, causal, -1, -1,
                   0.0, False, None, None)
        return r

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # Kernel-level timing with HIP events on the stream the kernels are launched on
    # (paged_attn launches on torch's current stream).
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.steps)]

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ev_ms = sum(s.elapsed_time(e) for s, e in evs) / a.steps

    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()

    flops_fwd = fwd_flops(B, H, S, S, D, causal)
    step_flops = flops_fwd * (3.5 if a.mode == "fwdbwd" else 1.0)
    value = step_flops * a.steps * world / elapsed / 1e12
    ms_per_step = elapsed / a.steps * 1e3

    allgather = None
    if dist:
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
        allgather = {"ms": round(ag_ms, 3), "bytes_per_rank_in": out.numel() * 2 * (world - 1),
                     "value_with_gather": round(step_flops * world / ((ms_per_step + ag_ms) / 1e3) / 1e12, 2)}

    if rank == 0:
        achieved = flops_fwd / (ev_ms / 1e3) / 1e12 if a.mode == "fwd" else step_flops / (ev_ms / 1e3) / 1e12
        line = {
            "metric": "attention TFLOPS/GPU (fwd, fwd+bwd) at S=4096 D=128; % MI355X MFMA peak",
            "value": round(value, 2),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (torch.randn, N(0,1)), inputs resident in HBM",
            "config": {"workload": f"mha_{a.mode} B={B} H={H} S={S} D={D} bf16 "
                                   f"{'causal' if causal else 'non-causal'}",
                       "global_batch": B * world, "seq_len": S, "heads": H, "head_dim": D,
                       "parallelism": f"dp{world} (batch x head shards, no collective in step)"},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 2),
                         "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": None,
                         "kernel_ms": round(ev_ms, 4)},
        }
        if allgather:
            line["allgather"] = allgather
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(8, S, D, causal, a.cpu_baseline_seconds)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""In-process A/B timing of kernel variants (interleaved rounds, one process, one device —
cdna_hip_programming.md §5.4 rule 24).

  python tools/perf_ab.py --opt fwd_waves=4,8 [--mode fwd|bwd|fwdbwd|fwd_fp8] [--rounds 5]
  python tools/perf_ab.py --var "" --var fwd_dyn=2 --var fwd_persistent=0   (whole variants)

Each variant's line also names the kernel and schedule it ran (fmha_last_kernel).
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", action="append", default=[], help="name=v1,v2,...")
    ap.add_argument("--var", action="append", default=[],
                    help="one whole variant: name=v,name=v ('' = the defaults); overrides --opt")
    ap.add_argument("--prewarm", type=float, default=1.0, help="untimed seconds first")
    ap.add_argument("--mode", default="fwd", choices=["fwd", "bwd", "fwdbwd", "fwd_fp8"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--b", type=int, default=4)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--hk", type=int, default=0)
    ap.add_argument("--s", type=int, default=4096)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--alibi", action="store_true", help="fwd: ALiBi slopes 2^-(8 (h+1) / H)")
    ap.add_argument("--softcap", type=float, default=0.0)
    ap.add_argument("--wl", type=int, default=-1, help="fwd: left window (with causal: a sliding window)")
    a = ap.parse_args()

    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    variants = [[]]
    for spec in a.opt:
        name, vals = spec.split("=")
        variants = [v + [(name, int(x))] for v in variants for x in vals.split(",")]
    if a.var:
        variants = [[(o.split("=")[0], int(o.split("=")[1])) for o in spec.split(",") if o]
                    for spec in a.var]
    defaults = {n: L.fmha_get_option(n.encode()) for vv in variants for n, _ in vv}
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    hk = a.hk or a.h
    causal = not a.noncausal
    q = torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=dt)
    k = torch.randn(a.b, a.s, hk, a.d, device="cuda", dtype=dt)
    v = torch.randn(a.b, a.s, hk, a.d, device="cuda", dtype=dt)
    do = torch.randn_like(q)
    out = torch.empty_like(q)
    pa = xfa.paged_attn
    sc = a.d ** -0.5
    lse = pa.fwd(q, k, v, out, None, 0.0, sc, causal, -1, -1, 0.0, False, None)[5]
    slopes = (2.0 ** (-8.0 * torch.arange(1, a.h + 1, device="cuda") / a.h)).float().expand(a.b, a.h).contiguous() \
        if a.alibi else None

    if a.mode == "fwd_fp8":
        def e4m3(t):                           # per-tensor scale to the e4m3 range (as bench.py)
            s8 = float(t.float().abs().max()) / 448.0
            return (t.float() / s8).to(torch.float8_e4m3fn), s8
        (q8, qs), (k8, ks), (v8, vs) = (e4m3(t) for t in (q, k, v))

    def run():
        if a.mode == "fwd_fp8":
            pa.fwd_fp8(q8, k8, v8, None, qs, ks, vs, sc, causal, -1, -1, False)
            return
        if a.mode in ("fwd", "fwdbwd"):
            pa.fwd(q, k, v, out, slopes, 0.0, sc, causal, a.wl, -1, a.softcap, False, None)
        if a.mode in ("bwd", "fwdbwd"):
            pa.bwd(do, q, k, v, out, lse, None, None, None, None, 0.0, sc, causal, -1, -1, 0.0,
                   False, None, None)

    fl = 4.0 * a.b * a.h * a.s * a.s * a.d * (0.5 if causal else 1.0)
    if a.wl >= 0 and causal:                   # visible pairs of a sliding window (wl, 0)
        w = min(a.wl, a.s - 1)
        fl = 4.0 * a.b * a.h * a.d * (a.s * (w + 1) - w * (w + 1) / 2)
    fl *= {"fwd": 1.0, "bwd": 2.5, "fwdbwd": 3.5, "fwd_fp8": 1.0}[a.mode]
    res = {str(vv): [] for vv in variants}
    kern = {}
    import time
    t = time.perf_counter()
    while time.perf_counter() - t < a.prewarm:
        run(); torch.cuda.synchronize()
    for r in range(a.rounds):
        for vv in variants:
            for name, val in defaults.items():
                assert L.fmha_set_option(name.encode(), val) == 0
            for name, val in vv:
                assert L.fmha_set_option(name.encode(), val) == 0, L.fmha_last_error()
            run(); torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                run()
            e.record(); torch.cuda.synchronize()
            res[str(vv)].append(s.elapsed_time(e) / a.iters)
            kern[str(vv)] = L.fmha_last_kernel().decode()
    for name, val in defaults.items():
        L.fmha_set_option(name.encode(), val)
    for vv, ts in res.items():
        med = statistics.median(ts)
        print(f"{a.mode} {vv}: median {med:.4f} ms  min {min(ts):.4f}  max {max(ts):.4f}  -> "
              f"{fl / med / 1e9:.1f} TFLOP/s  [{kern[vv]}]", flush=True)


if __name__ == "__main__":
    main()

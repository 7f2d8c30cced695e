"""PROBE harness: the 8-wave ping-pong forward (tools/gen_pingpong.py,
tools/probe/libpingpong.so) against the product's 4-wave kernel and its ablation builds, in one
process, interleaved rounds, on the C2 shape non-causal (B 4, H 32, S 4096, D 128 bf16; every
item has 64 key tiles, so no causal item-shape effect enters the comparison).

Per variant and round: 0.25 s of untimed launches (the clock settles to that variant's power),
then `iters` launches between HIP events; the GPU clock and socket power over the timed window
come from bench.py's side-process monitor (amd-smi).  Results of the timing variants marked
"INVALID" (ablations) are not checked; pp_full is checked against the product kernel.

  python tools/pingpong_ab.py [--rounds 5] [--iters 20] [--lib name=path ...]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import shutil
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", action="append", default=[],
                    help="name=path of an extra libpaged-attention build (e.g. an ablation)")
    ap.add_argument("--causal", action="store_true", help="product variants causal (pp is not)")
    ap.add_argument("--pp", action="append", default=[],
                    help="name=path of a ping-pong probe build (tools/probe/build.sh); default base")
    a = ap.parse_args()
    import bench
    mon = bench.ClockMonitor()                      # before this process touches the GPU
    try:
        run(a, mon)
    finally:
        mon.close()


def run(a, mon):
    import torch
    import bench
    mon.select(bench.device_info(torch.device("cuda", 0))["pci_bus"])
    from xf_flash_attention_cutlass_amd import capi
    B, S, H, D = 4, 4096, 32, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    o = torch.empty_like(q)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    stream = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    sc = D ** -0.5
    wr = 0 if a.causal else -1

    def product(lib):
        return lambda: lib.fmha_fwd(P(q), P(k), P(v), P(o), None, S, S, B, H, H, D, 0.0, stream,
                                    None, sc, None, P(lse), -1, wr, 0.0, False, False, 0)

    variants = []
    prod = capi.lib()
    variants.append(("4w (product)", product(prod)))
    tmp = os.path.join(tempfile.mkdtemp(), "lib_8w.so")
    shutil.copy(os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "lib", "libpaged-attention.so"), tmp)
    l8 = capi.load(tmp, strict=False)
    assert l8.fmha_set_option(b"fwd_w4", 0) == 0
    variants.append(("8w compiler-scheduled (fwd_w4=0)", product(l8)))
    for spec in a.lib:
        name, path = spec.split("=", 1)
        variants.append((name + " [INVALID: ablation]", product(capi.load(path, strict=False))))
    pps = []
    for spec in a.pp or ["base=" + os.path.join(ROOT, "tools", "probe", "libpp_base.so")]:
        name, path = spec.split("=", 1)
        lib = ctypes.CDLL(os.path.abspath(path))
        lib.pp_launch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 4 + [
            ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
        pps.append((name, lib))
    po = torch.empty_like(q)
    plse = torch.empty_like(lse)

    def pp_run(lib, full):
        def f():
            assert lib.pp_launch(P(q), P(k), P(v), P(po), P(plse), B, S, H, H, sc, full, stream) == 0
        return f
    for name, lib in pps:
        variants.append((f"pp skel {name} (MFMA+LDS+DMA+barriers) [INVALID]", pp_run(lib, 0)))
    for name, lib in pps:
        variants.append((f"pp full {name} (8-wave ping-pong)", pp_run(lib, 1)))

    # sanity: every full ping-pong against the product kernel (non-causal)
    prod.fmha_fwd(P(q), P(k), P(v), P(o), None, S, S, B, H, H, D, 0.0, stream, None, sc, None,
                  P(lse), -1, -1, 0.0, False, False, 0)
    for name, lib in pps:
        pp_run(lib, 1)()
        torch.cuda.synchronize()
        do = (po.float() - o.float()).abs().max().item()
        dl = (plse - lse).abs().max().item()
        print(f"check pp full {name} vs product (non-causal): max|dO| {do:.3e} "
              f"(|O|max {o.float().abs().max().item():.3f}), max|dLSE| {dl:.3e}", flush=True)

    fl = 4.0 * B * H * S * S * D * (0.5 if a.causal else 1.0)
    flpp = 4.0 * B * H * S * S * D
    res = {n: [] for n, _ in variants}
    win = {n: [] for n, _ in variants}
    t = time.time()
    while time.time() - t < 1.0:
        variants[0][1]()
        torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, f in variants:
            t0 = time.time()
            while time.time() - t0 < 0.25:
                for _ in range(4):
                    f()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            w0 = time.time()
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            win[name].append((w0 - 0.15, time.time()))
            res[name].append(e0.elapsed_time(e1) / a.iters)
    for name, _ in variants:
        med = statistics.median(res[name])
        flops = flpp if name.startswith("pp") else fl
        clk = [mon.stats(w0, w1) for w0, w1 in win[name]]
        mhz = [c["gfx_mhz_median"] for c in clk if c.get("samples")]
        pw = [c["power_w_median"] for c in clk if c.get("samples") and c.get("power_w_median")]
        mhz_s = f"{statistics.median(mhz):.0f} MHz" if mhz else "- MHz"
        pw_s = f"{statistics.median(pw):.0f} W" if pw else "- W"
        tf = flops / med / 1e9
        per_ghz = f"{tf / (statistics.median(mhz) / 1e3):.0f} TF/GHz" if mhz else ""
        print(f"{name:48s} median {med:.4f} ms (min {min(res[name]):.4f})  {tf:7.1f} TFLOP/s  "
              f"{mhz_s} {pw_s} {per_ghz}", flush=True)


if __name__ == "__main__":
    main()

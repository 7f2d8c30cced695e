"""Per-tile vs per-item cost of the forward kernel: non-causal, fixed items, varying key length
(tiles per item = Sk / 64); a least-squares fit t = items_per_cu * (a + b * tiles) separates
the main-loop cost per tile (b) from the fixed per-item cost (a: prologue, pipeline fill,
drain, O store).

  python tools/fwd_fit.py [--b 16] [--h 32] [--sq 512] [--sks 1024,2048,4096,8192]
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
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--sq", type=int, default=512)
    ap.add_argument("--sks", default="512,1024,2048,4096,8192")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import xf_flash_attention_cutlass_amd as xfa
    from xf_flash_attention_cutlass_amd import capi
    L = capi.lib()
    for spec in a.opt:
        n, v = spec.split("=")
        assert L.fmha_set_option(n.encode(), int(v)) == 0
    pa = xfa.paged_attn
    d = 128
    sc = d ** -0.5
    q = torch.randn(a.b, a.sq, a.h, d, device="cuda", dtype=torch.bfloat16)
    out = torch.empty_like(q)
    sks = [int(x) for x in a.sks.split(",")]
    kv = {sk: (torch.randn(a.b, sk, a.h, d, device="cuda", dtype=torch.bfloat16),
               torch.randn(a.b, sk, a.h, d, device="cuda", dtype=torch.bfloat16)) for sk in sks}
    # clock-ramp prewarm
    k, v = kv[sks[-1]]
    for _ in range(200):
        pa.fwd(q, k, v, out, None, 0.0, sc, False, -1, -1, 0.0, False, None)
    torch.cuda.synchronize()
    items = a.b * a.h * ((a.sq + 255) // 256)
    ipc = items / 256.0
    rows = []
    for rep in range(3):
        for sk in sks:
            k, v = kv[sk]
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.iters):
                pa.fwd(q, k, v, out, None, 0.0, sc, False, -1, -1, 0.0, False, None)
            s1.record()
            torch.cuda.synchronize()
            rows.append((sk, s0.elapsed_time(s1) / a.iters))
    med = {sk: statistics.median([t for s, t in rows if s == sk]) for sk in sks}
    xs = [sk / 64 for sk in sks]
    ys = [med[sk] * 1e3 / ipc for sk in sks]      # us per item per CU
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    a0 = my - b * mx
    for sk in sks:
        fl = 4.0 * a.b * a.h * a.sq * sk * d
        print(f"sk={sk:6d} tiles/item={sk // 64:4d} {med[sk]:.4f} ms {fl / med[sk] / 1e9:7.1f} TFLOP/s")
    print(f"fit: per tile {b:.3f} us, per item {a0:.3f} us (= {a0 / b:.1f} tiles); "
          f"loop-only rate {4.0 * 256 * 64 * d / (b * 1e-6) / 1e12 * 256:.1f} TFLOP/s")


if __name__ == "__main__":
    main()

"""In-process timing of the backward with float-atomic dQ vs the deterministic mode (bounded
dQ slices walked in key-block order) (same inputs, interleaved rounds).  python tools/bwd_det_ab.py [--s 4096] [--noncausal]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=4)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--s", type=int, default=4096)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import xf_flash_attention_cutlass_amd as xfa
    pa = xfa.paged_attn
    causal = not a.noncausal
    q, k, v, do = (torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    sc = a.d ** -0.5
    r = pa.fwd(q, k, v, None, None, 0.0, sc, causal, -1, -1, 0.0, False, None)
    out, lse = r[0], r[5]

    def run(det):
        return pa.bwd(do, q, k, v, out, lse, None, None, None, None, 0.0, sc, causal, -1, -1, 0.0,
                      det, None, None)
    g0, g1 = run(False), run(True)
    torch.cuda.synchronize()
    print("dq max diff", (g0[0].float() - g1[0].float()).abs().max().item(),
          "dk/dv equal", torch.equal(g0[1], g1[1]), torch.equal(g0[2], g1[2]))
    for _ in range(20):
        run(False)
    torch.cuda.synchronize()
    fl = 4.0 * a.b * a.h * a.s * a.s * a.d * (0.5 if causal else 1.0) * 2.5
    times = {False: [], True: []}
    for _ in range(a.rounds):
        for det in (False, True):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run(det)
            e1.record()
            torch.cuda.synchronize()
            times[det].append(e0.elapsed_time(e1) / a.iters)
    for det in (False, True):
        m = statistics.median(times[det])
        print(f"bwd deterministic={det}: median {m:.4f} ms -> {fl / m / 1e9:.1f} TFLOP/s (bwd only)")


if __name__ == "__main__":
    main()

"""Read the phase stamps of a diagnostic 4-wave fp8 build (gen_fwd8.py --stamps, built by
tools/fwd8_variant.py): per wave, the share of s_memtime cycles in each phase class over the
fp8 forward at the C2 shape (B4 H32 S4096 D128 e4m3fn, causal and non-causal).  Read the
SHARES: the stamps' own lgkmcnt(0) waits also retire the LDS reads a step leaves in flight,
so the build runs slower than the product (cdna_hip_programming.md §7).

  python tools/fwd8_stamps.py variants/lib_f8st.so [--iters 20]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gen_fwd8 import ST_NAMES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from xf_flash_attention_cutlass_amd import capi
    lib = capi.load(a.lib, strict=False)
    st = ctypes.CDLL(a.lib).fmha_fwd8_stamps
    st.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    b, h, s, d = 4, 32, 4096, 128
    xs = []                                  # bench.py workload_fp8's inputs: N(0, 1), scaled
    for _ in range(3):
        t = torch.randn(b, s, h, d, device="cuda")
        sc = float(t.abs().max()) / 448.0
        xs.append(((t / sc).to(torch.float8_e4m3fn), sc))
    (q, qs), (k, ks), (v, vs) = xs
    o = torch.empty(b, s, h, d, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(b, h, s, device="cuda", dtype=torch.float32)
    P = lambda t: t.data_ptr()  # noqa: E731
    stream = torch.cuda.current_stream().cuda_stream
    buf = (ctypes.c_ulonglong * 32)()
    for causal in (True, False):
        wr = 0 if causal else -1

        def run():
            lib.fmha_fwd_fp8(P(q), P(k), P(v), P(o), P(lse), qs, ks, vs, s, s, b, h, h, d, d ** -0.5,
                             -1, wr, False, stream)
        for _ in range(5):
            run()
        assert st(buf, 1) == 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.iters
        assert st(buf, 1) == 0
        print(f"\nC2 shape fp8 {'causal' if causal else 'non-causal'}, {a.iters} launches, "
              f"{ms:.4f} ms per launch (stamps build), kernel {lib.fmha_last_kernel().decode()}")
        print("| wave | " + " | ".join(ST_NAMES) + " | total Gcyc |")
        print("|---" * (len(ST_NAMES) + 2) + "|")
        tot_all = [0] * len(ST_NAMES)
        for w in range(4):
            vals = [buf[w * 8 + c] for c in range(len(ST_NAMES))]
            tot = sum(vals)
            tot_all = [x + y for x, y in zip(tot_all, vals)]
            print(f"| {w} | " + " | ".join(f"{100 * x / tot:.1f} %" for x in vals) + f" | {tot / 1e9:.2f} |")
        T = sum(tot_all)
        print("| all | " + " | ".join(f"{100 * x / T:.1f} %" for x in tot_all) + f" | {T / 1e9:.2f} |")


if __name__ == "__main__":
    main()

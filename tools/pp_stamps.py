"""Read the phase stamps of a diagnostic ping-pong build (gen_fwdpp.py --stamps, built by
tools/fwdpp_variants.sh "st=--stamps"): per wave, the share of s_memtime cycles in each phase
class over the C2 forward (B4 H32 S4096 D128, causal unless --noncausal).  Read the SHARES: the
stamps' own lgkmcnt(0) waits change the timing they measure (cdna_hip_programming.md §7).

  python tools/pp_stamps.py variants/lib_st.so [--noncausal] [--iters 20]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CLASSES = ["M run", "M->V wait", "V run", "V->M wait", "prologue", "tail", "epilogue"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--w4", type=int, default=2, help="fwd_w4: 2 the 32x32x16 body, 3 the 16x16x32 body")
    ap.add_argument("--wl", type=int, default=-1, help="left window (causal: a sliding window)")
    ap.add_argument("--iters", type=int, default=3,
                    help="launches summed (the device counters are 32-bit: keep 256 CUs x launches x cycles < 2^32)")
    a = ap.parse_args()
    from xf_flash_attention_cutlass_amd import capi
    lib = capi.load(a.lib, strict=False)
    assert lib.fmha_set_option(b"fwd_w4", a.w4) == 0
    st = ctypes.CDLL(a.lib).fmha_fwdpp_stamps
    st.argtypes = [ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
    b, h, s, d = 4, 32, 4096, 128
    q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    o = torch.empty_like(q)
    lse = torch.empty(b, h, s, device="cuda", dtype=torch.float32)
    wr = -1 if a.noncausal else 0
    P = lambda t: t.data_ptr()  # noqa: E731
    stream = torch.cuda.current_stream().cuda_stream

    def run():
        lib.fmha_fwd(P(q), P(k), P(v), P(o), None, s, s, b, h, h, d, 0.0, stream, None, d ** -0.5,
                     None, P(lse), a.wl, wr, 0.0, False, False, 0)
    buf = (ctypes.c_uint * 64)()
    for _ in range(5):
        run()
    assert st(buf, 1) == 0
    for _ in range(a.iters):
        run()
    assert st(buf, 1) == 0
    print(f"C2 {'non-causal' if a.noncausal else 'causal'} window left {a.wl}, {a.iters} launches, kernel {lib.fmha_last_kernel().decode()}")
    print("wave | " + " | ".join(CLASSES) + " | total Mcyc")
    for w in range(8):
        vals = [buf[w * 8 + c] for c in range(len(CLASSES))]
        tot = sum(vals)
        print(f"{w} | " + " | ".join(f"{100 * x / tot:.1f}%" for x in vals) + f" | {tot / 1e6:.1f}")


if __name__ == "__main__":
    main()

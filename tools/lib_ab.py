"""In-process A/B timing of DIFFERENT BUILDS of libpaged-attention.so through the C ABI
(interleaved rounds on one device, so box-to-box clock differences cancel;
cdna_hip_programming.md §5.4 rule 24).

  python tools/lib_ab.py libA.so libB.so [--mode fwd|bwd] [--rounds 5] [--noncausal]
  (a build spec may carry options: path@name=val,...; det=1 runs the backward deterministic)

Each path is loaded as its own ctypes library (copy it under a distinct file name first:
the dynamic loader dedups by soname/path).  Options (--opt name=value) apply to every build.
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--mode", default="fwd", choices=["fwd", "bwd", "fwd_fp8", "decode"])
    ap.add_argument("--ragged", action="store_true", help="decode: cache lengths U[1, 32768]")
    ap.add_argument("--bf16cache", action="store_true", help="decode: bf16 K/V cache instead of fp8")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--b", type=int, default=4)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--hk", type=int, default=0)
    ap.add_argument("--s", type=int, default=4096)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--wl", type=int, default=-1, help="fwd: left window (with causal: a sliding window)")
    a = ap.parse_args()

    from xf_flash_attention_cutlass_amd import capi
    # a build may be given as path@name=val,name=val: per-build options (the same .so under
    # two options is copied to a distinct name so each load has its own option state)
    import shutil
    import tempfile
    libs = []
    dets = []   # per build: bwd deterministic flag (pseudo-option det=1 in the spec)
    for i, spec in enumerate(a.libs):
        path, _, opts = spec.partition("@")
        det = any(x == "det=1" for x in opts.split(","))
        opts = ",".join(x for x in opts.split(",") if x and not x.startswith("det="))
        dets.append(det)
        if opts:
            tmp = os.path.join(tempfile.mkdtemp(), f"v{i}_" + os.path.basename(path))
            shutil.copy(path, tmp)
            path = tmp
        lib = capi.load(path, strict=False)
        for o in a.opt + ([x for x in opts.split(",") if x] if opts else []):
            name, val = o.split("=")
            assert lib.fmha_set_option(name.encode(), int(val)) == 0, lib.fmha_last_error()
        libs.append(lib)
    hk = a.hk or a.h
    causal = not a.noncausal
    dt = torch.bfloat16
    q = torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=dt)
    k = torch.randn(a.b, a.s, hk, a.d, device="cuda", dtype=dt)
    v = torch.randn(a.b, a.s, hk, a.d, device="cuda", dtype=dt)
    o = torch.empty_like(q)
    do = torch.randn_like(q)
    lse = torch.empty(a.b, a.h, a.s, device="cuda", dtype=torch.float32)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    sc = a.d ** -0.5
    wr = 0 if causal else -1
    stream = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731

    if a.mode == "fwd_fp8":
        q8, k8, v8 = (t.to(torch.float8_e4m3fn) for t in (q, k, v))
    if a.mode == "decode":
        # C5 per GPU: B 8, H 32, Hk 8, cache 32768 (fp8 e4m3fn, page 16, random block table)
        DB, DH, DHK, DS, page = 8, 32, 8, 32768, 16
        nb = DB * DS // page
        table = torch.randperm(nb, device="cuda").to(torch.int32).view(DB, DS // page)
        dq_ = torch.randn(DB, 1, DH, 128, device="cuda", dtype=dt)
        do_ = torch.empty_like(dq_)
        dlse = torch.empty(DB, DH, 1, device="cuda", dtype=torch.float32)
        lens = torch.full((DB,), DS, dtype=torch.int32, device="cuda")
        if a.ragged:
            lens = torch.randint(1, DS + 1, (DB,), generator=torch.Generator().manual_seed(0)).to(torch.int32).cuda()
        kvt = dt if a.bf16cache else torch.float8_e4m3fn
        kc = (torch.randn(nb, page, DHK, 128, device="cuda") * 4).to(kvt)
        vc = (torch.randn(nb, page, DHK, 128, device="cuda") * 4).to(kvt)
        o = do_
        dbytes = 2 * int(lens.sum()) * DHK * 128 * kc.element_size()

    def run(lib):
        det = dets[libs.index(lib)]
        if a.mode == "decode":
            lib.fmha_page_kvcache_fwd_ex(P(dq_), P(kc), P(vc), P(do_), P(dlse), P(table), DS // page,
                                         P(lens), 1, DS, DB, DH, DHK, 128, page, 128 ** -0.5, -1, 0,
                                         0.0, None, 0, 0, 0 if a.bf16cache else 1, 1.0, 1.0, None, False, stream)
            return
        if a.mode == "fwd_fp8":
            lib.fmha_fwd_fp8(P(q8), P(k8), P(v8), P(o), P(lse), 1.0, 1.0, 1.0, a.s, a.s, a.b, a.h,
                             hk, a.d, sc, -1, wr, False, stream)
            return
        lib.fmha_fwd(P(q), P(k), P(v), P(o), None, a.s, a.s, a.b, a.h, hk, a.d, 0.0, stream, None,
                     sc, None, P(lse), a.wl, wr, 0.0, False, False, 0)
        if a.mode == "bwd":
            lib.fmha_bwd(P(do), P(q), P(k), P(v), P(o), P(lse), P(dq), P(dk), P(dv), None, None,
                         a.s, a.s, a.b, a.h, hk, a.d, 0.0, sc, -1, wr, 0.0, det, False, stream,
                         None, 0)

    # outputs of every build against the first one's (atomic dQ sums differ in the last bits
    # from run to run, so this is a sanity check, not the parity test)
    ref = None
    for i, lib in enumerate(libs):
        for t in (o, dq, dk, dv):
            t.zero_()
        run(lib)
        torch.cuda.synchronize()
        outs = [t.float().clone() for t in ((o, dq, dk, dv) if a.mode == "bwd" else (o,))]
        if ref is None:
            ref = outs
            continue
        diffs = " ".join(f"{n}:{(x - r).abs().max().item():.3e}/{r.abs().max().item():.2e}"
                         for n, x, r in zip(("o", "dq", "dk", "dv"), outs, ref))
        print(f"check {os.path.basename(a.libs[i])} vs {os.path.basename(a.libs[0])}: {diffs}")

    fl = 4.0 * a.b * a.h * a.s * a.s * a.d * (0.5 if causal else 1.0) * (3.5 if a.mode == "bwd" else 1.0)
    for lib in libs:
        for _ in range(3):
            run(lib)
    torch.cuda.synchronize()
    # ~1 s clock-ramp prewarm (bench.py does the same)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 0
    while True:
        run(libs[0])
        n += 1
        if n % 20 == 0:
            e1.record()
            torch.cuda.synchronize()
            if e0.elapsed_time(e1) > 1000:
                break
    times = {i: [] for i in range(len(libs))}
    for _ in range(a.rounds):
        for i, lib in enumerate(libs):
            s0 = torch.cuda.Event(enable_timing=True)
            s1 = torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.iters):
                run(lib)
            s1.record()
            torch.cuda.synchronize()
            times[i].append(s0.elapsed_time(s1) / a.iters)
    for i, p in enumerate(a.libs):
        med = statistics.median(times[i])
        rate = (f"{dbytes / med / 1e9:.3f} TB/s" if a.mode == "decode" else f"{fl / med / 1e9:.1f} TFLOP/s")
        print(f"{a.mode} {os.path.basename(p)}: median {med:.4f} ms  min {min(times[i]):.4f}  -> {rate}")


if __name__ == "__main__":
    main()

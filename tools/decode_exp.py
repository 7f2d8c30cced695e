"""Decode kernel experiments (in-process): GB/s for page sizes, cache dtypes, split counts.
  python tools/decode_exp.py"""
import os, sys, statistics
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xf_flash_attention_cutlass_amd as xfa
pa = xfa.paged_attn
dev = "cuda"
B, H, HK, D, S = 8, 32, 8, 128, 32768


def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters)
    return statistics.median(ts)


def case(page, fp8, splits):
    nblk = S // page
    nb = B * nblk
    table = torch.randperm(nb, device=dev).to(torch.int32).view(B, nblk)
    esz = 1 if fp8 else 2
    if fp8:
        kc = (torch.randn(nb, page, HK, D, device=dev) * 4).to(torch.float8_e4m3fn).view(torch.uint8)
        vc = (torch.randn(nb, page, HK, D, device=dev) * 4).to(torch.float8_e4m3fn).view(torch.uint8)
    else:
        kc = torch.randn(nb, page, HK, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn(nb, page, HK, D, device=dev, dtype=torch.bfloat16)
    q = torch.randn(B, 1, H, D, device=dev, dtype=torch.bfloat16)
    lens = torch.full((B,), S, dtype=torch.int32, device=dev)
    if fp8:
        fn = lambda: pa.fwd_kvcache_fp8(q, kc, vc, lens, table, 0.25, 0.25, D ** -0.5, False, -1, -1, splits)
    else:
        fn = lambda: pa.fwd_kvcache(q, kc, vc, None, None, lens, None, None, None, table, None, None,
                                    D ** -0.5, False, -1, -1, 0.0, True, splits)
    ms = timeit(fn)
    gb = B * S * HK * D * 2 * esz / 1e9
    print(f"page={page:4d} {'fp8 ' if fp8 else 'bf16'} splits={splits:3d}: {ms*1e3:7.1f} us  {gb/ms*1e3:7.1f} GB/s", flush=True)
    del kc, vc


for fp8 in (True, False):
    for page in (16, 256):
        for splits in (0, 16, 64, 128):
            case(page, fp8, splits)

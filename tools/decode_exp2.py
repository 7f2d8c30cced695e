"""Decode bandwidth hypotheses: kv-head interleaving, batch, dense vs paged."""
import os, sys, statistics
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xf_flash_attention_cutlass_amd as xfa
from xf_flash_attention_cutlass_amd import capi
pa = xfa.paged_attn
dev = "cuda"
D = 128


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


def dense(B, H, HK, S, splits=0):
    q = torch.randn(B, 1, H, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(B, S, HK, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(B, S, HK, D, device=dev, dtype=torch.bfloat16)
    o = torch.empty_like(q)
    lse = torch.empty(B, H, 1, device=dev)
    L = capi.lib()
    fn = lambda: L.fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, 1, S, B, H, HK, D,
                            0.0, capi.stream_handle(), None, D ** -0.5, None, lse.data_ptr(), -1, -1, 0.0,
                            False, False, splits)
    ms = timeit(fn)
    gb = B * S * HK * D * 2 * 2 / 1e9
    print(f"dense bf16 B={B} H={H} HK={HK} S={S} splits={splits}: {ms*1e3:7.1f} us {gb/ms*1e3:7.1f} GB/s", flush=True)


dense(8, 32, 8, 32768)
dense(8, 32, 1, 32768 * 8)
dense(64, 32, 8, 4096)
dense(64, 32, 8, 32768 // 2)
dense(8, 32, 8, 32768, 128)
dense(8, 8, 8, 32768)

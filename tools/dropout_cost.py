"""Cost of dropout at the C2/C3 shape (B4 H32 S4096 D128 bf16 causal): forward and
forward+backward with p = 0 and p = 0.1, medians of event-timed rounds on one device."""
import os, statistics, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xf_flash_attention_cutlass_amd as xfa

B, H, S, D = 4, 32, 4096, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
           for _ in range(3))
g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
fl = 4.0 * B * H * S * S * D * 0.5


def fwd(p):
    with torch.no_grad():
        xfa.flash_attn_func(q, k, v, dropout_p=p, causal=True)


def fwdbwd(p):
    o = xfa.flash_attn_func(q, k, v, dropout_p=p, causal=True)
    torch.autograd.grad(o, (q, k, v), g)


for name, fn, mult in (("fwd", fwd, 1.0), ("fwd+bwd", fwdbwd, 3.5)):
    res = {}
    for p in (0.0, 0.1):
        for _ in range(5):
            fn(p)
    torch.cuda.synchronize()
    for r in range(5):
        for p in (0.0, 0.1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn(p)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(p, []).append(e0.elapsed_time(e1) / 10)
    for p, ts in res.items():
        ms = statistics.median(ts)
        print(f"{name} p={p}: {ms:.3f} ms  {fl * mult / ms / 1e9:.0f} TFLOP/s")

"""In-process A/B of decode options on the C5 shape (per GPU: B=8 H=32 Hk=8, cache 32768,
page 16, fp8 or bf16 K/V): python tools/decode_ab.py --opt fwd_decode16=0,1 [--bf16]"""
import argparse, os, statistics, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--opt", action="append", default=[])
ap.add_argument("--bf16", action="store_true")
ap.add_argument("--ragged", action="store_true", help="cache lengths U[1, S] (bench.py --ragged)")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
import xf_flash_attention_cutlass_amd as xfa
from xf_flash_attention_cutlass_amd import capi
L = capi.lib()
pa = xfa.paged_attn
B, H, HK, D, S, page = 8, 32, 8, 128, 32768, 16
nb = B * S // page
table = torch.randperm(nb, device="cuda").to(torch.int32).view(B, S // page)
q = torch.randn(B, 1, H, D, device="cuda", dtype=torch.bfloat16)
lens = torch.full((B,), S, dtype=torch.int32, device="cuda")
if a.ragged:
    lens = torch.randint(1, S + 1, (B,), generator=torch.Generator().manual_seed(0)).to(torch.int32).cuda()
if a.bf16:
    kc = torch.randn(nb, page, HK, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(nb, page, HK, D, device="cuda", dtype=torch.bfloat16)
    run = lambda: xfa.flash_attn_with_kvcache(q, kc, vc, cache_seqlens=lens, block_table=table)
    nbytes = 2 * int(lens.sum()) * HK * D * 2
else:
    kc = (torch.randn(nb, page, HK, D, device="cuda") * 4).to(torch.float8_e4m3fn).view(torch.uint8)
    vc = (torch.randn(nb, page, HK, D, device="cuda") * 4).to(torch.float8_e4m3fn).view(torch.uint8)
    run = lambda: pa.fwd_kvcache_fp8(q, kc, vc, lens, table, 0.25, 0.25, D ** -0.5, False, -1, -1, 0)
    nbytes = 2 * int(lens.sum()) * HK * D
variants = [[]]
for spec in a.opt:
    n, vals = spec.split("=")
    variants = [v + [(n, int(x))] for v in variants for x in vals.split(",")]
for _ in range(50):
    run()
torch.cuda.synchronize()
res = {str(v): [] for v in variants}
outs = {}
for r in range(a.rounds):
    for v in variants:
        for n, x in v:
            L.fmha_set_option(n.encode(), x)
        o = run(); torch.cuda.synchronize()
        outs[str(v)] = (o[0] if isinstance(o, (tuple, list)) else o).float().clone()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.iters):
            run()
        s1.record(); torch.cuda.synchronize()
        res[str(v)].append(s0.elapsed_time(s1) / a.iters)
base = outs[str(variants[0])]
for v, ts in res.items():
    med = statistics.median(ts)
    print(f"{v}: median {med * 1e3:.1f} us  -> {nbytes / med / 1e6:.0f} GB/s (step incl. combine)  max|o - o[{variants[0]}]| = {(outs[v] - base).abs().max().item():.3g}")

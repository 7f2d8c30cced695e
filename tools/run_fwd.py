"""Run one attention kernel configuration a few times (for rocprofv3 --pmc / --kernel-trace).
  python tools/run_fwd.py [--opt name=v ...] [--mode fwd|bwd] [--iters N] [--noncausal]"""
import argparse, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--opt", action="append", default=[])
ap.add_argument("--mode", default="fwd")
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--noncausal", action="store_true")
ap.add_argument("--b", type=int, default=4); ap.add_argument("--h", type=int, default=32)
ap.add_argument("--s", type=int, default=4096); ap.add_argument("--d", type=int, default=128)
a = ap.parse_args()
import xf_flash_attention_cutlass_amd as xfa
from xf_flash_attention_cutlass_amd import capi
for o in a.opt:
    n, v = o.split("="); assert capi.lib().fmha_set_option(n.encode(), int(v)) == 0
q = torch.randn(a.b, a.s, a.h, a.d, device="cuda", dtype=torch.bfloat16)
k, v, do = torch.randn_like(q), torch.randn_like(q), torch.randn_like(q)
out = torch.empty_like(q)
c = not a.noncausal
r = xfa.paged_attn.fwd(q, k, v, out, None, 0.0, a.d ** -0.5, c, -1, -1, 0.0, False, None)
for _ in range(a.iters):
    if a.mode == "fwd":
        xfa.paged_attn.fwd(q, k, v, out, None, 0.0, a.d ** -0.5, c, -1, -1, 0.0, False, None)
    else:
        xfa.paged_attn.bwd(do, q, k, v, out, r[5], None, None, None, None, 0.0, a.d ** -0.5, c,
                           -1, -1, 0.0, False, None, None)
torch.cuda.synchronize()

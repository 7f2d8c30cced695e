import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xf_flash_attention_cutlass_amd as xfa
pa = xfa.paged_attn
B, H, HK, D, S, page = 8, 32, 8, 128, 32768, 16
nb = B * S // page
table = torch.randperm(nb, device="cuda").to(torch.int32).view(B, S // page)
kc = (torch.randn(nb, page, HK, D, device="cuda") * 4).to(torch.float8_e4m3fn).view(torch.uint8)
vc = (torch.randn(nb, page, HK, D, device="cuda") * 4).to(torch.float8_e4m3fn).view(torch.uint8)
q = torch.randn(B, 1, H, D, device="cuda", dtype=torch.bfloat16)
lens = torch.full((B,), S, dtype=torch.int32, device="cuda")
for _ in range(4):
    pa.fwd_kvcache_fp8(q, kc, vc, lens, table, 0.25, 0.25, D ** -0.5, False, -1, -1, 0)
torch.cuda.synchronize()

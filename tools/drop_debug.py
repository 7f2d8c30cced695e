"""Dropout debug: per (batch, head) error of the forward against the oracle given the mask."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xf_flash_attention_cutlass_amd as xfa
from oracle import attention_ref as orc
for (b, h, hk, sq, sk, d, causal) in ((2, 4, 2, 128, 128, 128, True), (1, 1, 1, 128, 128, 128, True),
                                      (1, 2, 2, 64, 64, 128, False), (2, 1, 1, 64, 64, 128, False),
                                      (1, 2, 1, 64, 64, 128, False)):
    torch.manual_seed(2)
    p = 0.2
    q = torch.randn(b, sq, h, d, dtype=torch.bfloat16)
    k = torch.randn(b, sk, hk, d, dtype=torch.bfloat16)
    v = torch.randn(b, sk, hk, d, dtype=torch.bfloat16)
    for api in ("raw", "func"):
        if api == "raw":
            r = xfa.paged_attn.fwd(q.cuda(), k.cuda(), v.cuda(), None, None, p, d ** -0.5, causal, -1, -1, 0.0, True, None)
            out, s = r[0], r[6]
        else:
            out, lse, s = xfa.flash_attn_func(q.cuda(), k.cuda(), v.cuda(), dropout_p=p, causal=causal, return_attn_probs=True)
        out, s = out.float().cpu(), s.float().cpu()
        mask = ~torch.signbit(s[:, :, :sq, :sk])
        o, attn = orc.attention_ref(q, k, v, None, None, None, p, mask, causal=causal)
        e = (out - o.float()).abs().amax(dim=(1, 3))  # [b, h]
        print((b, h, hk, sq, sk, causal), api, "err[b,h]", [[round(x, 4) for x in row] for row in e.tolist()],
              "S-attn", (s[:, :, :sq, :sk].abs() - attn.float()).abs().max().item())

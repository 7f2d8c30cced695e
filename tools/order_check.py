import torch, sys
sys.path.insert(0, '.')
import xf_flash_attention_cutlass_amd as xfa
from xf_flash_attention_cutlass_amd import capi
L = capi.lib()
pa = xfa.paged_attn
torch.manual_seed(0)
for (b,h,hk,s,causal) in [(4,32,32,4096,True),(2,16,4,3000,True),(3,8,8,1000,False),(1,64,8,8192,True)]:
    q = torch.randn(b,s,h,128,device='cuda',dtype=torch.bfloat16)
    k = torch.randn(b,s,hk,128,device='cuda',dtype=torch.bfloat16)
    v = torch.randn(b,s,hk,128,device='cuda',dtype=torch.bfloat16)
    outs=[]
    for o in (0,1):
        assert L.fmha_set_option(b"fwd_order", o) == 0
        out = torch.empty_like(q)
        r = pa.fwd(q,k,v,out,None,0.0,128**-0.5,causal,-1,-1,0.0,False,None)
        torch.cuda.synchronize()
        outs.append((out.clone(), r[5].clone()))
    print(b,h,hk,s,causal, torch.equal(outs[0][0],outs[1][0]), torch.equal(outs[0][1],outs[1][1]))

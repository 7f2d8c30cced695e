"""Where a 4-wave forward workgroup's time goes: inside the item bodies (the asm pipeline) vs
the C++ item setup around them, from a diagnostics build (-DXFA_FWD4_STAMP, s_memtime stamps).

  python tools/quick_variant.py stamp "-DXFA_FWD4_STAMP" fwd:128:bf16
  python tools/fwd4_stamp.py variants/lib_stamp.so
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from xf_flash_attention_cutlass_amd import capi
    lib = capi.load(sys.argv[1], strict=False)
    rd = lib.fmha_fwd4_stamp_bf16
    buf = (ctypes.c_ulonglong * 4)()
    b, s, h, d = 4, 4096, 32, 128
    q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    o = torch.empty_like(q)
    lse = torch.empty(b, h, s, device="cuda", dtype=torch.float32)
    st = torch.cuda.current_stream().cuda_stream
    for causal in (True, False):
        wr = 0 if causal else -1
        for _ in range(5):
            lib.fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, s, s, b, h, h, d,
                         0.0, st, None, d ** -0.5, None, lse.data_ptr(), -1, wr, 0.0, False, False, 1)
        torch.cuda.synchronize()
        rd(buf)
        n = 20
        for _ in range(n):
            lib.fmha_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), None, s, s, b, h, h, d,
                         0.0, st, None, d ** -0.5, None, lse.data_ptr(), -1, wr, 0.0, False, False, 1)
        torch.cuda.synchronize()
        rd(buf)
        t_in, tot, waves = buf[0], buf[1], buf[2]
        items = b * h * (s // 256) * n           # per launch x launches (one per workgroup)
        per_wave_items = items * 4 / waves
        print(f"{'causal' if causal else 'noncausal'}: inside item bodies {t_in / tot:.3f} of wave time; "
              f"outside per item {(tot - t_in) / waves / per_wave_items:.0f} cycles "
              f"(s_memtime ticks), per item inside {t_in / waves / per_wave_items:.0f}", flush=True)


if __name__ == "__main__":
    main()

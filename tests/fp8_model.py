"""Numerics model of this build's 4-wave fp8 forward (test-only; csrc/fmha_fwd8w_kernel.h,
tools/gen_fwd8.py): the same arithmetic as oracle.attention_fp8_pt except for WHICH maximum P is
taken against before its e4m3 rounding.

The estimate (attention_fp8_pt) rounds P = exp(s - rowmax) with the row's true maximum, so the
row's largest term is exactly 1.0, which e4m3 represents exactly.  The kernel keeps no row max in
its loop: P = 2^(s c - m) against m = the masked max of key tile 0, and only when a lane's partial
row sum of a tile passes 2^slack (any lane of the 64-row wave) does the wave take the rare path
(m = max(m, the tile's max), O and l rescaled, the tile redone).  So the kernel's largest terms
sit anywhere in [1, 2^8] and take e4m3's rounding error (up to 2^-4 relative) where the estimate
takes none; in peaked rows (large scores) that term dominates the output.  This model repeats the
kernel's reference maxima, its wave grouping (64 GQA-packed rows of a 256-row item) and its
lane-half partial sums, so the kernel's error can be compared with the error of its own
arithmetic.  Not a parity oracle: nothing of the reference is involved.
"""
from __future__ import annotations

import math

import torch

from oracle import attention_ref as orc


def attention_fp8_kernel_model(q8, k8, v8, q_scale, k_scale, v_scale, causal=False,
                               window_size=(-1, -1), slack=8):
    """fp32 [b, sq, h, d] output of the 4-wave fp8 kernel's arithmetic (see the module doc)."""
    b, sq, h, d = q8.shape
    sk, hk = k8.shape[1], k8.shape[2]
    G = h // hk
    q, k, v = (x.float() * s for x, s in ((q8, q_scale), (k8, k_scale), (v8, v_scale)))
    if causal:
        window_size = (window_size[0], 0)
    masked = orc.local_mask(sq, sk, window_size) if (window_size[0] >= 0 or window_size[1] >= 0) \
        else torch.zeros(sq, sk, dtype=torch.bool)
    c = d ** -0.5 * math.log2(math.e)
    thr = 2.0 ** min(slack, 8)
    half = ((torch.arange(64) >> 2) & 1).bool()          # key 32 kt + 8 d + 4 hh + i: lane half hh
    out = torch.zeros(b, sq, h, d)
    ntile = (sk + 63) // 64
    for bi in range(b):
        for kh in range(hk):
            rows = sq * G                                  # GQA packing: row = pos G + g
            qp = q[bi, :, kh * G:(kh + 1) * G].reshape(rows, d).double()
            pos = torch.arange(rows) // G
            s_all = (qp @ k[bi, :, kh].double().T) * c     # log2 units
            vis_all = ~masked[pos]
            vv = v[bi, :, kh]
            o_rows = torch.zeros(rows, d)
            for w0 in range(0, rows, 64):
                sw, vis = s_all[w0:w0 + 64], vis_all[w0:w0 + 64]
                n = sw.shape[0]
                seen = vis.any(0).nonzero()
                if seen.numel() == 0:
                    continue
                t_w = int(seen.max()) // 64                 # the wave's last key tile
                m0 = torch.where(vis[:, :64], sw[:, :64], torch.tensor(-math.inf)).amax(1)
                m = torch.where(torch.isfinite(m0), m0, torch.zeros_like(m0))
                L = torch.zeros(n, dtype=torch.float64)
                O = torch.zeros(n, d)
                for t in range(min(t_w + 1, ntile)):
                    st, vt = sw[:, 64 * t:64 * t + 64], vis[:, 64 * t:64 * t + 64]
                    hf = half[:st.shape[1]]
                    P = torch.where(vt, torch.exp2(st - m[:, None]), torch.zeros_like(st))
                    if t > 0:
                        lt = torch.stack([P[:, ~hf].sum(1), P[:, hf].sum(1)])
                        if bool((lt > thr).any()):         # wave-uniform rare path
                            mx = torch.where(vt, st, torch.tensor(-math.inf)).amax(1)
                            mn = torch.maximum(m, mx)
                            alpha = torch.exp2(m - mn)
                            O *= alpha[:, None].float()
                            L *= alpha
                            m = mn
                            P = torch.where(vt, torch.exp2(st - m[:, None]), torch.zeros_like(st))
                    L += P.sum(1)
                    p8 = P.float().to(torch.float8_e4m3fn).float()
                    O += p8 @ vv[64 * t:64 * t + st.shape[1]]
                o_rows[w0:w0 + n] = torch.where(L[:, None] > 0, O / L[:, None].float(), torch.zeros_like(O))
            out[bi, :, kh * G:(kh + 1) * G] = o_rows.view(sq, G, d)
    return out

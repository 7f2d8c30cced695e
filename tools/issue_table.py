"""Per-step issue-cost table of a generated forward body.

Takes the first asm statement of a generated body (the bf16-output instance), the steady-state
unmasked step between two labels, classifies its instructions and prices each class with the
issue costs measured in MI355X_MICROARCH.md (constants table, "vector-instruction ISSUE cost"
and "LDS-DMA piece"): transcendental 8 cycles, other VALU 4, s_nop N max(4, N+1), an MFMA
holds its SIMD's issue 8 cycles, an LDS-DMA piece ~60 among MFMAs.  The MFMA pipe time of the
step is given beside the issue total: a step whose issue total (one wave per SIMD) or whose
VALU phase (ping-pong: the partner wave's MFMAs run meanwhile) exceeds it is issue-bound.

  python tools/issue_table.py [--md out.md]
"""
from __future__ import annotations

import argparse
import os
import re
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc")

# (body, step start label, step end label, MFMA pipe cycles per MFMA, description)
BODIES = [
    ("fmha_fwd8_body.h", ".Lph1_%=:", ".Lnx1_%=:", 64, "fp8 4-wave (fp8_w4=1, default): one wave/SIMD, 64 rows x 64 keys"),
    ("fmha_fwd8pp_body.h", ".Lph1_A_%=:", ".Lnx1_A_%=:", 64, "fp8 ping-pong (fp8_w4=2): one wave's M + V phase, 32 rows x 64 keys"),
    ("fmha_fwdpp_body.h", ".Lph1_A_%=:", ".Lnx1_A_%=:", 32, "bf16 ping-pong (fwd_w4=2, default): one wave's M + V phase, 32 rows x 64 keys"),
    ("fmha_fwd4_body.h", ".Lph1_%=:", ".Lnx1_%=:", 32, "bf16 4-wave (fwd_w4=1): one wave/SIMD, 64 rows x 64 keys"),
]
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def step_lines(body, start, end):
    text = open(os.path.join(CSRC, body)).read()
    first = text.split("asm volatile(", 2)[1]
    lines = [m.group(1) for m in re.finditer(r'^\s*"(.*)\\n"\s*$', first, re.M)]
    i = lines.index(start)
    j = lines.index(end, i)
    return lines[i + 1:j]


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "MFMA", 8
    if op.startswith("buffer_load") and ins.rstrip().endswith("lds"):
        return "LDS-DMA piece", 60
    if op.startswith(TRANS):
        return "VALU transcendental (" + op + ")", 8
    if op.startswith("v_"):
        return "VALU " + op, 4
    if op.startswith("ds_read"):
        return "LDS read " + op, 4
    if op == "s_nop":
        n = int(ins.split()[1])
        return f"s_nop {n}", max(4, n + 1)
    if op in ("s_waitcnt", "s_barrier"):
        return op, 0
    if op.startswith("s_"):
        return "SALU / branch", 1
    return op, 4


def table(body, start, end, mfma_cyc, desc):
    ins = [x for x in step_lines(body, start, end) if x and not x.startswith(".")]
    cnt, cost = Counter(), {}
    for x in ins:
        k, c = classify(x)
        cnt[k] += 1
        cost[k] = c
    n_mfma = cnt.get("MFMA", 0)
    rows = sorted(cnt, key=lambda k: -cnt[k] * cost[k])
    total = sum(cnt[k] * cost[k] for k in cnt)
    valu = sum(cnt[k] * cost[k] for k in cnt if k.startswith("VALU") or k.startswith("s_nop"))
    out = [f"### `{body}` — {desc}", "",
           f"step = `{start[:-1]}` … `{end[:-1]}` of the bf16-output instance: {len(ins)} instructions, "
           f"{n_mfma} MFMAs = **{n_mfma * mfma_cyc} MFMA pipe cycles**; issue total ≈ **{total}** cycles "
           f"(VALU + nops {valu}).", "",
           "| class | count | issue cycles each | cycles |", "|---|---|---|---|"]
    for k in rows:
        out.append(f"| {k} | {cnt[k]} | {cost[k]} | {cnt[k] * cost[k]} |")
    return out + [""]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    out = ["# Per-step issue-cost tables of the generated forward bodies (`tools/issue_table.py`)", "",
           "Costs: MI355X_MICROARCH.md constants table (transcendental 8, VALU 4, an MFMA holds issue 8, "
           "LDS-DMA piece ~60 among MFMAs, s_nop N max(4, N+1); waits and barriers priced 0 — their cost "
           "is stall, not issue). Static counts of the steady-state unmasked step.", ""]
    for b in BODIES:
        out += table(*b)
    text = "\n".join(out)
    if a.md:
        open(a.md, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()

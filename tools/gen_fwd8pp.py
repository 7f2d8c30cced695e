"""Generate csrc/fmha_fwd8pp_body.h: the 8-wave ping-pong fp8 (e4m3fn) forward body
(csrc/fmha_fwd8pp_kernel.h).

The phase program of tools/gen_fwdpp.py (read its docstring: two waves per SIMD, waves 4-7 one
phase behind waves 0-3, MFMA phases PV(j) + QK^T(j+1) against VALU phases softmax(j+1) +
LDS-DMA, the unmasked / masked / last / idle step variants, the rare redo path) on the operand
layouts of the 4-wave fp8 kernel (tools/gen_fwd8.py): both GEMMs on the block-scaled
v_mfma_scale_f32_32x32x64_f8f6f4 (E8M0 scales 1.0, 64 cycles per MFMA), a wave of 32 query rows
per 64-key tile runs 4 QK^T + 4 PV MFMAs (512 cycles) against its 32 scores' softmax, which is
where the 4-wave fp8 kernel spent its time (VALU-bound): here the partner wave's
MFMAs run beside it.

This module imports gen_fwdpp and rebinds its operand-specific pieces (fragment reads, MFMAs,
P packing, DMA pieces, Q loads, wait states, the v_scale epilogue factor), so the phase logic
itself exists once.

Register map (per lane, 256 = v[0:127] + a[0:127]):
  a[0:63]    O^T accumulators (4 d tiles x 16)
  a[64:79]   Q fragments (2 x 8: d 0-63, 64-127; 32 bytes per lane each)
  a[80:111]  K fragment ring (4 slots x 8: one tile's (kt, s) fragments)
  v[0:31]    S;  v[32:39] P (8 dwords of e4m3, the B operand of PV with the k permutation of
             gen_fwd8.py);  v[40:47] scratch;  v48 tile row sum, v49 -m, v50 running sum,
  v51 key limit, v52-55 redo / max temps, v56 = 127 (E8M0 scale 1.0)
  v[64:95]   V^T fragment ring (4 slots x 8)

  python tools/gen_fwd8pp.py       (writes xf_flash_attention_cutlass_amd/csrc/fmha_fwd8pp_body.h)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fwdpp as pp  # noqa: E402

pp.FEATURES = False    # (no softcap / ALiBi pass in this body)
pp.LEFTWIN = False     # (no left windows: the one-sided key limit)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc", "fmha_fwd8pp_body.h")

TILE = 64 * 128        # one fp8 K (or V) tile
MNEM = "v_mfma_scale_f32_32x32x64_f8f6f4"
SC127 = 56
ABASE_Q, ABASE_K, VBASE_V = 64, 80, 64
LEAD = 4               # gaps a K fragment read leads its MFMA

pp.SBASE, pp.PBASE, pp.TMP = 0, 32, 40
pp.LT, pp.NM, pp.LRUN, pp.LIM, pp.MISC = 48, 49, 50, 51, 52
# the 32x32x64 fp8 MFMA's results: 40 wait states before a VALU reads them (gen_fwd8.py)
pp.XDL_NOPS = ["s_nop 7"] * 5
pp.VPH_NOPS = ["s_nop 7"] * 5
pp.NPIECE = 2          # one K and one V piece per wave and tile (8 KiB tiles, 8 waves)
pp.EPI_SCALE = "%[vsc]"


def qtup(s):
    return f"a[{ABASE_Q + 8 * s}:{ABASE_Q + 8 * s + 7}]"


def ktup(slot, half=None):
    b = ABASE_K + 8 * slot
    return f"a[{b}:{b + 7}]" if half is None else f"a[{b + 4 * half}:{b + 4 * half + 3}]"


def vtup(slot, kb=None):
    b = VBASE_V + 8 * slot
    return f"v[{b}:{b + 7}]" if kb is None else f"v[{b + 2 * kb}:{b + 2 * kb + 1}]"


def value_info(v):
    """score v (kt*16 + r): key offset in the tile minus 4*hh, P dword (4 e4m3 per dword)"""
    kt, r = v // 16, v % 16
    return 32 * kt + 8 * (r >> 2) + (r & 3), 4 * kt + (r >> 2)


def softmax(dt, mask):
    """P = e4m3(exp2(S c - m)) of this lane's 32 scores, fp32 row sum in LT (gen_fwd8.py's ops)"""
    ops = []
    for v in range(32):
        t = f"v{pp.TMP + v % 8}"
        off, dword = value_info(v)
        ex = [f"v_exp_f32 {t}, {t}"]
        if mask:
            ex += [f"v_cmp_lt_i32 vcc, {off}, v{pp.LIM}", f"v_cndmask_b32 {t}, 0, {t}, vcc"]
        st = [[f"v_fma_f32 {t}, v{pp.SBASE + v}, %[c], v{pp.NM}"], ex,
              [f"v_mov_b32 v{pp.LT}, {t}" if v == 0 else f"v_add_f32 v{pp.LT}, v{pp.LT}, {t}"]]
        if v & 1:
            sel = " op_sel:[0,0,1]" if (v % 16) & 3 == 3 else ""
            st[2].append(f"v_cvt_pk_fp8_f32 v{pp.PBASE + dword}, v{pp.TMP + (v - 1) % 8}, {t}{sel}")
        for k, txt in enumerate(st):
            ops.append((v + 2 * k, v, txt))
    out = []
    for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1])):
        out += txt
    return out + ["s_nop 0"]


def k_reads(f, slot_tile):
    kt, s = f // 2, f % 2
    return [f"ds_read_b128 {ktup(f, u)}, %[ka{2 * s + u}] offset:{slot_tile * TILE + kt * 32 * 128}"
            for u in (0, 1)]


def v_reads(dt_, slot_tile):
    return [f"ds_read_b64_tr_b8 {vtup(dt_, kb)}, %[va{dt_}] offset:{slot_tile * TILE + kb * 2048}"
            for kb in range(4)]


def m_phase(dt, j_slot, pv=True, qk=True):
    """PV(j) (4 MFMAs) then QK^T(j+1) (4 MFMAs); with qk, tile j+1's 4 V^T fragments are read at
    the end (the next PV's operands).  On entry with pv, this tile's V^T fragments (16 reads)
    are the only LDS reads in flight."""
    sc = f"v{SC127}, v{SC127} op_sel_hi:[0,0,0]"
    nx = (j_slot + 1) % pp.RING
    mf = []
    if pv:
        for d in range(4):
            mf.append((("V", d), f"{MNEM} {pp.otup(d)}, {vtup(d)}, v[{pp.PBASE}:{pp.PBASE + 7}], {pp.otup(d)}, {sc}"))
    if qk:
        for f in range(4):
            kt, s = f // 2, f % 2
            acc = pp.sv(kt)
            mf.append((("K", f), f"{MNEM} {acc}, {ktup(f)}, {qtup(s)}, {acc if s else '0'}, {sc}"))
    G = len(mf)
    first, last = {}, {}
    for g, (tag, _) in enumerate(mf):
        first.setdefault(tag, g)
        last[tag] = g
    reads = []
    if qk:
        for f in range(4):
            g = max(first[("K", f)] - LEAD, 0) if first[("K", f)] > 0 else -1
            reads.append((g, 0, k_reads(f, nx), ("K", f)))
        for d in range(4):
            lo = (last[("V", d)] + 2) if pv else 0
            g = max(lo, G - 8 + 2 * d)
            reads.append((min(g, G), 2 + d, v_reads(d, nx), ("N", d)))
    issued, last_idx = [], {}
    if pv:
        for d in range(4):
            issued += [("V", d)] * 4
            last_idx[("V", d)] = len(issued) - 1
    waited = 0
    byg = {}
    for g, o, txt, tag in reads:
        byg.setdefault(g, []).append((o, txt, tag))
    out = []
    for g in range(-1, G + 1):
        for o, txt, tag in sorted(byg.get(g, []), key=lambda x: x[0]):
            out += txt
            issued += [tag] * len(txt)
            if tag[0] in "KV":
                last_idx[tag] = len(issued) - 1
        if 0 <= g < G:
            tag, text = mf[g]
            if tag in last_idx and last_idx[tag] >= waited:
                n = min(len(issued) - last_idx[tag] - 1, 15)
                out.append(f"s_waitcnt lgkmcnt({n})")
                waited = len(issued) - n
            out.append(text)
    return out


def dma_pieces(slot):
    """this wave's K piece and V piece of the tile in slot (8 rows x 128 bytes each)"""
    out = []
    for op, srd, base in (("dk", pp.SKR, 0), ("dv", pp.SVR, pp.RING * TILE)):
        out.append([f"s_add_u32 m0, %[kdst], {base + slot * TILE}", "s_nop 0",
                    f"buffer_load_dwordx4 %[{op}], s[{srd}:{srd + 3}], 0 offen lds"])
    return out


def item_program(dt):
    out = ["s_waitcnt lgkmcnt(0)",
           f"v_mov_b32 v{pp.NM}, 0", f"v_mov_b32 v{pp.LRUN}, 0", f"v_mov_b32 v{pp.LIM}, %[lim]",
           f"v_mov_b32 v{SC127}, 0x7f", f"s_mov_b32 s{pp.SST}, 0"]
    # Q fragments: s -> 2 x 16 bytes at d = 64 s + 32 hh (+ 16)
    for s in range(2):
        for u in range(2):
            b = ABASE_Q + 8 * s + 4 * u
            out.append(f"buffer_load_dwordx4 a[{b}:{b + 3}], %[qoff], %[qsrd], 0 offen offset:{64 * s + 16 * u}")
    out += [f"v_accvgpr_write_b32 a{pp.ABASE_O + i}, 0" for i in range(64)]
    for r, lo, hi in ((pp.SKR, "kblo", "kbhi"), (pp.SVR, "vblo", "vbhi")):
        out += [f"s_mov_b32 s{r}, %[{lo}]", f"s_mov_b32 s{r + 1}, %[{hi}]",
                f"s_mov_b32 s{r + 2}, %[kvbytes]", f"s_mov_b32 s{r + 3}, 0x20000"]
    for slot in range(pp.DLEAD - 1):                         # tiles 0 .. DLEAD-2
        out += sum(dma_pieces(slot), []) + pp.dma_advance()
    # Q and tile 0 landed, published
    out += [f"s_waitcnt vmcnt({pp.NPIECE * (pp.DLEAD - 2)})", "s_barrier"]
    out += ["s_cmp_eq_u32 %[grp], 0", "s_cbranch_scc0 .LgrpB_%="]
    out += pp.group_program(dt, 0) + [".LgrpB_%=:"] + pp.group_program(dt, 1) + [".Lend_%=:"]
    return out


pp.value_info = value_info
pp.softmax = softmax
pp.m_phase = m_phase
pp.dma_pieces = dma_pieces

SIG = ("const int kblo, const int kbhi, const int vblo, const int vbhi, const int kvbytes, "
       "const i32x4 qsrd, const i32x4 osrd, const i32x4 lsrd, const int kstep, const int kdst, "
       "const int ntl, const int tw, const int ew, const int grp, const float c, const float thr, "
       "const float vsc, const int ka0, const int ka1, const int ka2, const int ka3, const int va0, "
       "const int va1, const int va2, const int va3, const int dk, const int dv, const int lim, "
       "const int qoff, const int ooff, const int loff")
SOPS = ["kblo", "kbhi", "vblo", "vbhi", "kvbytes", "qsrd", "osrd", "lsrd", "kstep", "kdst", "ntl",
        "tw", "ew", "grp", "c", "thr", "vsc"]
VOPS = ["ka0", "ka1", "ka2", "ka3", "va0", "va1", "va2", "va3", "dk", "dv", "lim", "qoff", "ooff",
        "loff"]


def emit(out=OUT):
    lines = [
        "// GENERATED by tools/gen_fwd8pp.py -- do not edit by hand.",
        "// The 8-wave ping-pong fp8 forward's item body (fmha_fwd8pp_kernel.h): one asm statement",
        "// per output dtype with a fixed register map; see the generators' docstrings.",
        "#pragma once",
        '#include "fmha_common.h"',
        "",
        "namespace xfa {",
        "typedef __attribute__((ext_vector_type(4))) int i32x4;",
        f"constexpr int kFwd8ppRing = {pp.RING};          // K / V tile slots the body addresses",
        "",
    ]
    ops = [f'[{o}] "s"({o})' for o in SOPS] + [f'[{o}] "v"({o})' for o in VOPS]
    for dt in ("bf16", "f16"):
        prog = item_program(dt) + pp.GUARDS
        pp.GUARDS.clear()
        lines.append(f"__device__ __forceinline__ void fwd8pp_item_{dt}({SIG}) {{")
        lines.append("    asm volatile(")
        lines += [f'        "{b}\\n"' for b in prog]
        lines.append("        :")
        lines.append("        : " + ",\n          ".join(ops))
        lines.append(f"        : {pp.clobbers()});")
        lines.append("}")
        lines.append("")
        print(dt, len(prog), "instructions/labels")
    lines.append("}  // namespace xfa")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--abl", default="", help="timing ablations, comma list (results invalid)")
    ap.add_argument("--out", default=OUT)
    a = ap.parse_args()
    pp.ABL = set(x for x in a.abl.split(",") if x)
    emit(a.out)

"""Generate csrc/fmha_fwdpp16_body.h: the 8-wave ping-pong D = 128 forward body on the bf16 /
f16 MFMA shape v_mfma_f32_16x16x32 (csrc/fmha_fwdpp_kernel.h with M16).

The phase program of tools/gen_fwdpp.py (read its docstring: two waves per SIMD, waves 4-7 one
phase behind waves 0-3, MFMA phases PV(j) + QK^T(j+1) against VALU phases softmax(j+1) +
LDS-DMA, the unmasked / masked / last / idle step variants, the rare redo path) with the same
output tile per wave (32 query rows x 64 keys per step) on the 16x16x32 shape.  Why: at the
1.4 kW board cap the chip holds a higher clock on 16x16x32 than on 32x32x16 at equal cycles per
FLOP (MI355X_MICROARCH.md DVFS give-back item 7; probe tools/gen_pingpong16.py: +5 % per
second on the full ping-pong, +6 % clock).  Like gen_fwd8pp.py this module imports gen_fwdpp
and rebinds its operand-specific pieces, so the phase logic itself exists once.

Layout per wave (its 32 query rows = two 16-row tiles rt; g = lane >> 4, l16 = lane & 15):
  S^T(kt, rt) = K(kt) Q^T(rt)   16 keys x 16 rows over 4 k-steps of 32 d; a lane holds row
                                16 rt + l16 and keys 16 kt + 4 g + r (r = 0..3)   32 MFMAs
  O^T(dt, rt) += V^T(dt) P^T    16 d x 16 rows over 2 k-steps of 32 keys; k index m of lane
                                group g = key 32 ks + 16 (m >> 2) + 4 g + (m & 3): P(ks, rt) is
                                cvt_pk of S^T(2 ks, rt), S^T(2 ks + 1, rt) as they stand, the
                                V^T fragment two ds_read_b64_tr_b16 blocks 16 keys apart  32 MFMAs
  K fragment (kt, s): ds_read_b128 at kv_off(16 kt + l16, 4 s + g) (one base register)
  a row's 64 keys of a tile sit on the 4 lanes l16 + 16 g: row max / row sum reductions take a
  permlane32 and a permlane16 swap; each lane carries two rows (limit, -m, sums per row)

Register map (per lane, 256 = v[0:127] + a[0:127]):
  a[0:63]    O^T (8 dt x 2 rt x 4)         a[64:95]  Q (2 rt x 4 s x 4)
  a[96:127]  K fragment ring (8 x 4)
  v[0:31]    S (v = 8 kt + 4 rt + r)       v[32:47]  P (2 ks x 2 rt x 4 packed pairs)
  v[48:55]   softmax scratch               v[64:95]  V^T fragment ring (8 x 4)
  v56/57 tile row sums (rt 0 / 1), v58/59 -m, v60/61 running row sums, v62/63 key limits
  v[96:103]  max / redo temps

  python tools/gen_fwdpp16.py      (writes xf_flash_attention_cutlass_amd/csrc/fmha_fwdpp16_body.h)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fwdpp as pp  # noqa: E402

pp.FEATURES = False    # (no softcap / ALiBi pass in this body)
pp.LEFTWIN = False     # (no left windows: the one-sided key limit)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc", "fmha_fwdpp16_body.h")

TILE = pp.TILE
LEAD = 6               # MFMA gaps (16x16x32: half the 32x32x16 cycles) an LDS read leads its MFMA
pp.SBASE, pp.PBASE, pp.TMP = 0, 32, 48
LT, NM, LRUN, LIM, MISC = 56, 58, 60, 62, 96      # pairs: register + rt
pp.LT, pp.NM, pp.LRUN, pp.LIM, pp.MISC = LT, NM, LRUN, LIM, MISC
ABASE_O, ABASE_Q, ABASE_K, VBASE_V = 0, 64, 96, 64
pp.N_EPI_STORES = 18   # 16 O stores (8 bytes) + 2 LSE stores


def otup(dt, rt):
    b = ABASE_O + 4 * (2 * dt + rt)
    return f"a[{b}:{b + 3}]"


def qtup(rt, s):
    b = ABASE_Q + 4 * (4 * rt + s)
    return f"a[{b}:{b + 3}]"


def ktup(slot):
    return f"a[{ABASE_K + 4 * slot}:{ABASE_K + 4 * slot + 3}]"


def vtup(slot, half=None):
    b = VBASE_V + 4 * slot
    return f"v[{b}:{b + 3}]" if half is None else f"v[{b + 2 * half}:{b + 2 * half + 1}]"


def sv(kt, rt):
    b = pp.SBASE + 4 * (2 * kt + rt)
    return f"v[{b}:{b + 3}]"


def ptup(ks, rt):
    b = pp.PBASE + 4 * (2 * ks + rt)
    return f"v[{b}:{b + 3}]"


def value_info(v):
    """score v = 8 kt + 4 rt + r of this lane (its S register): key offset in the tile minus
    4 g, its row tile, P dword (pairs r, r + 1)"""
    kt, rt, r = v // 8, (v // 4) % 2, v % 4
    return 16 * kt + r, rt, pp.PBASE + 4 * (2 * (kt // 2) + rt) + 2 * (kt % 2) + r // 2


def k_read(f, slot_tile, dst_slot):
    s, kt = f // 4, f % 4
    return f"ds_read_b128 {ktup(dst_slot)}, %[kb0] offset:{slot_tile * TILE + 4096 * kt + 512 * s}"


def v_reads(f, slot_tile, dst_slot):
    ks, dt = f // 8, f % 8
    off = slot_tile * TILE + 8192 * ks + 512 * (dt >> 1)   # (the lane base carries the V ring)
    return [f"ds_read_b64_tr_b16 {vtup(dst_slot, h)}, %[vb{dt & 1}] offset:{off + 4096 * h}" for h in (0, 1)]


def m_phase(dt, j_slot, pv=True, qk=True):
    """PV(j) then QK^T(j+1) (j_slot = j mod RING); each K / V^T fragment feeds the MFMAs of both
    row tiles; with qk the next PV's first NVPRE V^T fragments (tile j+1) are read at the end.
    (gen_fwdpp.m_phase's read placement and lgkmcnt accounting over this MFMA list)"""
    mnem = "v_mfma_f32_16x16x32_" + dt
    nx = (j_slot + 1) % pp.RING
    KS, VS, NVPRE = pp.KS, pp.VS, pp.NVPRE
    mf = []
    if pv:
        for f in range(16):
            ks, d = f // 8, f % 8
            for rt in (0, 1):
                mf.append((("V", f), f"{mnem} {otup(d, rt)}, {vtup(f % VS)}, {ptup(ks, rt)}, {otup(d, rt)}"))
    if qk:
        for f in range(16):
            s, kt = f // 4, f % 4
            for rt in (0, 1):
                src = sv(kt, rt) if s else "0"
                mf.append((("K", f), f"{mnem} {sv(kt, rt)}, {ktup(f % KS)}, {qtup(rt, s)}, {src}"))
    G = len(mf)
    first, last = {}, {}
    for g, (tag, _) in enumerate(mf):
        first.setdefault(tag, g)
        last[tag] = g
    reads = []
    if pv:
        for f in range(NVPRE, 16):
            lo = last[("V", f - VS)] + 2 if f >= VS else 0
            g = min(max(lo, first[("V", f)] - LEAD, 0), first[("V", f)] - 1)
            reads.append((g, 1, v_reads(f, j_slot, f % VS), ("V", f)))
    if qk:
        for f in range(16):
            g = max(first[("K", f)] - LEAD, 0)
            if f >= KS:
                g = max(g, last[("K", f - KS)] + 2)
            g = min(g, first[("K", f)] - 1) if first[("K", f)] > 0 else -1
            reads.append((g, 0, [k_read(f, nx, f % KS)], ("K", f)))
        for f in range(NVPRE):
            lo = (last[("V", 16 - VS + f)] + 2) if pv else 0
            g = max(lo, G - 4 * NVPRE + 4 * f)
            reads.append((min(g, G), 2 + f, v_reads(f, nx, f), ("N", f)))
    issued, last_idx = [], {}
    if pv:
        for f in range(NVPRE):
            issued += [("V", f)] * 2
            last_idx[("V", f)] = len(issued) - 1
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


def softmax(dt, mask):
    """P = exp2(S c - m_rt) of this lane's 32 scores (2 rows x 16 keys; masked: keys at or past
    the row's limit give 0), the rows' tile sums in LT, LT + 1; 4 scores in flight"""
    ops = []
    started = [False, False]
    for v in range(32):
        t = f"v{pp.TMP + v % 8}"
        off, rt, dword = value_info(v)
        ex = [f"v_exp_f32 {t}, {t}"]
        if mask:
            ex += [f"v_cmp_lt_i32 vcc, {off}, v{LIM + rt}", f"v_cndmask_b32 {t}, 0, {t}, vcc"]
        acc = (f"v_add_f32 v{LT + rt}, v{LT + rt}, {t}" if started[rt] else f"v_mov_b32 v{LT + rt}, {t}")
        started[rt] = True
        st = [[f"v_fma_f32 {t}, v{pp.SBASE + v}, %[c], v{NM + rt}"], ex, [acc]]
        if v & 1:
            st[2].append(f"v_cvt_pk_{dt}_f32 v{dword}, v{pp.TMP + (v - 1) % 8}, {t}")
        for k, txt in enumerate(st):
            ops.append((v + 2 * k, v, txt))
    out = []
    for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1])):
        out += txt
    return out + ["s_nop 0"]


def row_reduce(op, dst, t2):
    """dst = op over the 4 lanes l16 + 16 g of this lane's row (permlane32 then permlane16)"""
    return [f"v_mov_b32 {t2}, {dst}", "s_nop 1", f"v_permlane32_swap_b32 {dst}, {t2}", "s_nop 1",
            f"{op} {dst}, {dst}, {t2}", f"v_mov_b32 {t2}, {dst}", "s_nop 1",
            f"v_permlane16_swap_b32 {dst}, {t2}", "s_nop 1", f"{op} {dst}, {dst}, {t2}"]


def row_max2(dst0, dst1):
    """masked max of each of the lane's two rows over the tile's 64 keys -> dst0, dst1"""
    t2, ninf = f"v{MISC + 2}", f"v{MISC + 5}"
    dst = (dst0, dst1)
    out = [f"v_mov_b32 {ninf}, 0xff800000", f"v_mov_b32 {dst0}, {ninf}", f"v_mov_b32 {dst1}, {ninf}"]
    for v in range(32):
        off, rt, _ = value_info(v)
        out += [f"v_cmp_lt_i32 vcc, {off}, v{LIM + rt}",
                f"v_cndmask_b32 {t2}, {ninf}, v{pp.SBASE + v}, vcc",
                f"v_max_f32 {dst[rt]}, {dst[rt]}, {t2}"]
    return out + row_reduce("v_max_f32", dst0, t2) + row_reduce("v_max_f32", dst1, t2)


def first_max():
    """m_rt = the masked max of tile 0 per row (NM = -c max, 0 for a row with no key)"""
    mx, t2 = f"v{MISC}", f"v{MISC + 2}"
    out = pp.XDL_NOPS + row_max2(mx, f"v{MISC + 1}")
    for rt in (0, 1):
        m = f"v{MISC + rt}"
        out += [f"v_mul_f32_e64 {t2}, -%[c], {m}", f"v_cmp_lg_f32 vcc, 0xff800000, {m}",
                f"v_cndmask_b32 v{NM + rt}, 0, {t2}, vcc"]
    return out


def redo_block(dt, uid):
    """rare path (gen_fwdpp.redo_block per row): the tile's true masked max per row, m_new =
    max(m, c max); the row's O and l scaled by 2^(m - m_new); the softmax redone"""
    out = [f".Lredo_{uid}:"] + pp.XDL_NOPS + row_max2(f"v{MISC}", f"v{MISC + 1}")
    t2 = f"v{MISC + 2}"
    alpha = (f"v{MISC + 3}", f"v{MISC + 4}")
    for rt in (0, 1):
        mx = f"v{MISC + rt}"
        out += [f"v_mul_f32 {t2}, %[c], {mx}",
                f"v_max_f32_e64 {t2}, {t2}, -v{NM + rt}",
                f"v_add_f32 {alpha[rt]}, v{NM + rt}, {t2}",
                f"v_exp_f32_e64 {alpha[rt]}, -{alpha[rt]}",
                f"v_mul_f32 v{NM + rt}, -1.0, {t2}",
                "s_nop 0",
                f"v_mul_f32 v{LRUN + rt}, v{LRUN + rt}, {alpha[rt]}"]
    for i in range(64):
        t = f"v{pp.TMP + i % 8}"
        rt = (i // 4) % 2
        out += [f"v_accvgpr_read_b32 {t}, a{ABASE_O + i}", f"v_mul_f32 {t}, {t}, {alpha[rt]}",
                f"v_accvgpr_write_b32 a{ABASE_O + i}, {t}"]
    out += ["s_nop 1"] + softmax(dt, True)
    return out + ["s_nop 3", f"s_setpc_b64 s[{pp.SRA}:{pp.SRA + 1}]"]


def redo_check(uid, tag):
    """(inline part, stub): either row's tile sum on any lane past 2^slack -> the rare path;
    then l += LT per row"""
    t = f"v{MISC + 2}"
    inline = [f"v_max_f32 {t}, v{LT}, v{LT + 1}", f"v_cmp_lt_f32 vcc, %[thr], {t}", "s_nop 1",
              f"s_cbranch_vccnz .Lrc{tag}_{uid}", f".Lnr{tag}_{uid}:",
              f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}", f"v_add_f32 v{LRUN + 1}, v{LRUN + 1}, v{LT + 1}"]
    stub = [f".Lrc{tag}_{uid}:", f"s_getpc_b64 s[{pp.SRA}:{pp.SRA + 1}]", f".Lpc{tag}_{uid}:",
            f"s_add_u32 s{pp.SRA}, s{pp.SRA}, .Lnr{tag}_{uid} - .Lpc{tag}_{uid}",
            *pp.addc_ret(pp.SRA + 1, f".Lnr{tag}_{uid}", f".Lpc{tag}_{uid}", True),
            f"s_branch .Lredo_{uid}"]
    return inline, stub


LIM_STEP = [f"v_add_u32 v{LIM}, -64, v{LIM}", f"v_add_u32 v{LIM + 1}, -64, v{LIM + 1}"]


def v_phase(dt, slot, kind, uid, tag):
    """gen_fwdpp.v_phase with both rows' key limits stepped"""
    pieces = pp.dma_pieces(slot)
    if kind == "n":
        return sum(pieces, []) + pp.dma_advance() + LIM_STEP, []
    sm = softmax(dt, kind == "m")
    out = pieces[0] + pp.VPH_NOPS
    step = len(sm) // len(pieces)
    for n, pc in enumerate(pieces[1:]):
        at = (n + 1) * step + 3 * n
        sm[at:at] = pc
    out += sm
    inl, stub = redo_check(uid, tag)
    out += inl + pp.dma_advance() + LIM_STEP
    return out, stub


def epilogue_core(dt):
    """per row: the sums of its 4 lanes combined, O / l -> dt (4 consecutive d per lane: 8-byte
    stores), LSE by the g = 0 lanes (loff is out of range on the others)"""
    T = pp.TMP
    inv = (f"v{T + 6}", f"v{T + 7}")
    out = []
    for rt in (0, 1):
        L, t, lse, cls, pinf = (f"v{T + i}" for i in range(5))
        out += [f"v_mov_b32 {pinf}, 0x7f800000", f"v_mov_b32 {L}, v{LRUN + rt}"]
        out += row_reduce("v_add_f32", L, t)
        out += [f"v_rcp_f32 {inv[rt]}, {L}", f"v_log_f32 {lse}, {L}",
                f"v_mov_b32 {cls}, 0x63", f"v_cmp_class_f32 vcc, {L}, {cls}",
                f"v_cndmask_b32_e64 {inv[rt]}, {inv[rt]}, 1.0, vcc",
                f"v_sub_f32 {lse}, {lse}, v{NM + rt}",
                f"v_mul_f32 {lse}, 0x3f317218, {lse}", f"v_cndmask_b32 {lse}, {lse}, {pinf}, vcc",
                f"buffer_store_dword {lse}, %[loff{rt}], %[lsrd], 0 offen"]
    for d in range(8):
        for rt in (0, 1):
            vb = 8 * ((2 * d + rt) % 4)                 # four rotating register sets in S
            vals = [f"v{vb + k}" for k in range(4)]
            src = [f"a{ABASE_O + 4 * (2 * d + rt) + k}" for k in range(4)]
            out += [f"v_accvgpr_read_b32 {vals[k]}, {src[k]}" for k in range(4)]
            out += [f"v_mul_f32 {vals[k]}, {vals[k]}, {inv[rt]}" for k in range(4)]
            out += [f"v_cvt_pk_{dt}_f32 v{vb + 4 + k}, {vals[2 * k]}, {vals[2 * k + 1]}" for k in range(2)]
            out += [f"buffer_store_dwordx2 v[{vb + 4}:{vb + 5}], %[ooff{rt}], %[osrd], 0 offen offset:{32 * d}"]
    return out


def item_program(dt):
    out = (["s_memtime s[96:97]", "s_waitcnt lgkmcnt(0)", "s_mov_b32 s98, s96"] if pp.STAMPS else [])
    out += ["s_waitcnt lgkmcnt(0)"]
    for rt in (0, 1):
        out += [f"v_mov_b32 v{NM + rt}, 0", f"v_mov_b32 v{LRUN + rt}, 0", f"v_mov_b32 v{LIM + rt}, %[lim{rt}]"]
    out += [f"s_mov_b32 s{pp.SST}, 0"]
    out += [f"buffer_load_dwordx4 {qtup(rt, s)}, %[qoff{rt}], %[qsrd], 0 offen offset:{64 * s}"
            for rt in (0, 1) for s in range(4)]
    out += [f"v_accvgpr_write_b32 a{ABASE_O + i}, 0" for i in range(64)]
    for r, lo, hi in ((pp.SKR, "kblo", "kbhi"), (pp.SVR, "vblo", "vbhi")):
        out += [f"s_mov_b32 s{r}, %[{lo}]", f"s_mov_b32 s{r + 1}, %[{hi}]",
                f"s_mov_b32 s{r + 2}, %[kvbytes]", f"s_mov_b32 s{r + 3}, 0x20000"]
    for slot in range(pp.DLEAD - 1):                         # tiles 0 .. DLEAD-2
        out += sum(pp.dma_pieces(slot), []) + pp.dma_advance()
    out += [f"s_waitcnt vmcnt({pp.NPIECE * (pp.DLEAD - 2)})", "s_barrier"]   # Q and tile 0 landed
    out += ["s_cmp_eq_u32 %[grp], 0", "s_cbranch_scc0 .LgrpB_%="]
    out += pp.group_program(dt, 0) + [".LgrpB_%=:"] + pp.group_program(dt, 1) + [".Lend_%=:"]
    return out


SIG = ("const int kblo, const int kbhi, const int vblo, const int vbhi, const int kvbytes, "
       "const i32x4 qsrd, const i32x4 osrd, const i32x4 lsrd, const int kstep, const int kdst, "
       "const int ntl, const int tw, const int ew, const int grp, const float c, const float thr, "
       "const int kb0, const int vb0, const int vb1, const int dma0, const int dma1, "
       "const int lim0, const int lim1, const int qoff0, const int qoff1, const int ooff0, "
       "const int ooff1, const int loff0, const int loff1")
OPS = ['[kblo] "s"(kblo)', '[kbhi] "s"(kbhi)', '[vblo] "s"(vblo)', '[vbhi] "s"(vbhi)',
       '[kvbytes] "s"(kvbytes)', '[qsrd] "s"(qsrd)', '[osrd] "s"(osrd)', '[lsrd] "s"(lsrd)',
       '[kstep] "s"(kstep)', '[kdst] "s"(kdst)', '[ntl] "s"(ntl)', '[tw] "s"(tw)', '[ew] "s"(ew)',
       '[grp] "s"(grp)', '[c] "s"(c)', '[thr] "s"(thr)',
       '[kb0] "v"(kb0)', '[vb0] "v"(vb0)', '[vb1] "v"(vb1)',
       '[dma0] "v"(dma0)', '[dma1] "v"(dma1)', '[lim0] "v"(lim0)', '[lim1] "v"(lim1)',
       '[qoff0] "v"(qoff0)', '[qoff1] "v"(qoff1)', '[ooff0] "v"(ooff0)', '[ooff1] "v"(ooff1)',
       '[loff0] "v"(loff0)', '[loff1] "v"(loff1)']


def clobbers():
    regs = [f'"v{i}"' for i in range(MISC + 8)] + [f'"a{i}"' for i in range(128)]
    regs += [f'"s{i}"' for i in range(pp.SKR, pp.SCM + 2)] + \
        ([f'"s{i}"' for i in range(96, 100)] if pp.STAMPS else [])
    return ", ".join(regs + ['"vcc"', '"scc"', '"memory"'])


# the phase program's operand-specific pieces, rebound
pp.m_phase, pp.softmax, pp.first_max, pp.redo_block = m_phase, softmax, first_max, redo_block
pp.redo_check, pp.v_phase, pp.epilogue_core = redo_check, v_phase, epilogue_core


def emit(out=OUT):
    lines = [
        "// GENERATED by tools/gen_fwdpp16.py -- do not edit by hand.",
        "// The 8-wave ping-pong D = 128 forward's item body on v_mfma_f32_16x16x32 (fmha_fwdpp_kernel.h,",
        "// M16): one asm statement per dtype with a fixed register map; see the generator's docstring.",
        "#pragma once",
        '#include "fmha_common.h"',
        "",
        *(["#define XFA_FWDPP16_STAMPS 1         // diagnostic build (--stamps)"] if pp.STAMPS else []),
        "namespace xfa {",
        "typedef __attribute__((ext_vector_type(4))) int i32x4;",
        f"constexpr int kFwdpp16Ring = {pp.RING};         // K / V tile slots the body addresses",
        "",
    ]
    for dt in ("bf16", "f16"):
        prog = item_program(dt)
        prog += pp.GUARDS
        pp.GUARDS.clear()
        sig = SIG + (", unsigned& acc" if pp.STAMPS else "")
        lines.append(f"__device__ __forceinline__ void fwdpp16_item_{dt}({sig}) {{")
        lines.append("    asm volatile(")
        lines += [f'        "{b}\\n"' for b in prog]
        lines.append('        : [acc] "+v"(acc)' if pp.STAMPS else "        :")
        lines.append("        : " + ",\n          ".join(OPS))
        lines.append(f"        : {clobbers()});")
        lines.append("}")
        lines.append("")
        print(dt, len(prog), "instructions/labels")
    lines.append("}  // namespace xfa")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--lead", type=int, default=LEAD)
    ap.add_argument("--stamps", action="store_true", help="diagnostic phase stamps")
    ap.add_argument("--out", default=OUT)
    a = ap.parse_args()
    LEAD = a.lead
    pp.STAMPS = a.stamps
    emit(a.out)

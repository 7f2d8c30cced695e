"""Probe generator: an 8-wave "ping-pong" D = 128 forward, two waves per SIMD.

NOT part of the product.  It answers one question with a measurement: does a second wave per
SIMD, running its LDS-DMA issue and softmax VALU while its partner issues MFMAs, beat the
4-wave kernel (one wave per SIMD, everything on one instruction stream)?

Structure (tools/probe/pingpong.hip wraps the generated item body):
  * workgroup = 8 waves x 32 query rows = 256 rows (the 4-wave kernel's item), waves w and w+4
    on one SIMD; group A = waves 0-3, group B = waves 4-7;
  * per wave and 64-key tile: an MFMA phase M(j) = PV(j) then QK^T(j+1) (32 x
    v_mfma_f32_32x32x16, K / V^T fragments from LDS in the gaps), and a VALU phase V(j) =
    softmax(j+1) (fma, exp, add per score, cvt per pair) + the wave's 4 LDS-DMA pieces of tile
    j+3; every phase ends at an s_barrier, and group B runs one phase behind group A, so on each
    SIMD one wave is in its MFMA phase while the other is in its VALU phase;
  * K / V tiles in 4-slot LDS rings (the kv_off image of the 4-wave kernel); tile t is published
    at the barrier ending global phase 2t-1 (A: s_waitcnt vmcnt(4) after its V phase, B:
    vmcnt(0) after its M phase);
  * probe simplification: no running max (P = exp2(S c), exact for N(0,1) inputs, whose scores
    stay far from fp32 overflow); the row sums and the output are real (pingpong_ab.py checks
    the full variant against torch);
  * mode "skel": the VALU phase keeps only the DMA (MFMA + LDS reads + DMA + barriers), the
    verdict's skeleton.

Register map per wave (256 = v[0:127] + a[0:127]):
  a[0:63] O^T (4 x 16), a[64:95] Q (8 x 4), a[96:127] K fragment ring (8 slots)
  v[0:31] S (2 x 16), v[32:47] P (4 x 4), v[48:55] scratch (epilogue temps), v[56:57] tile row
  sums, v58 running row sum, v59 -m (0), v[60:61] (c, c), v[62:63] (-m, -m), v[64:95] V^T
  fragment ring (8 slots)

  python tools/gen_pingpong.py     -> tools/probe/pingpong_body.h
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "probe", "pingpong_body.h")

HD = 128
RB = HD * 16           # one 8-row block of the kv_off image
TILE = 64 * HD * 2     # one K (or V) tile
VREG = 4 * TILE        # V ring after the 4 K slots
KS, VS = 8, 8          # fragment ring slots
LEAD = 6               # gaps an LDS read leads its MFMA
NVPRE = 4              # V^T fragments of the next M phase read at the end of this one
SBASE, PBASE, TMP = 0, 32, 48
LT, LRUN, NM, CP, NMP = 56, 58, 59, 60, 62   # LT: v[56:57] partial row sums; CP, NMP: (c, c), (-m, -m)
PK = True              # softmax on packed fp32 (v_pk_fma_f32, v_pk_add_f32): half the fma / add
DMAMIX = True          # the VALU phase's 4 DMA pieces spread through the softmax
LAST = True            # the last step peeled: no QK^T / softmax of the tile past the end
ABASE_O, ABASE_Q, ABASE_K, VBASE_V = 0, 64, 96, 64
SKR, SVR = 80, 84      # DMA descriptors (next tile to load), K and V
SRA = 92


def otup(d):
    return f"a[{ABASE_O + 16 * d}:{ABASE_O + 16 * d + 15}]"


def qtup(s):
    return f"a[{ABASE_Q + 4 * s}:{ABASE_Q + 4 * s + 3}]"


def ktup(slot):
    return f"a[{ABASE_K + 4 * slot}:{ABASE_K + 4 * slot + 3}]"


def vtup(slot, half=None):
    b = VBASE_V + 4 * slot
    return f"v[{b}:{b + 3}]" if half is None else f"v[{b + 2 * half}:{b + 2 * half + 1}]"


def sv(kt):
    return f"v[{SBASE + 16 * kt}:{SBASE + 16 * kt + 15}]"


def ptup(ks):
    return f"v[{PBASE + 4 * ks}:{PBASE + 4 * ks + 3}]"


def value_info(v):
    """score v (kt*16 + r): key offset in the tile minus 4*hh, P dword"""
    kt, r = v // 16, v % 16
    off = 32 * kt + 8 * (r >> 2) + (r & 3)
    ks = 2 * kt + (r >> 3)
    return off, ks * 4 + ((r & 7) >> 1)


def k_read(f, slot_tile, dst_slot):
    s, kt = f // 2, f % 2
    return f"ds_read_b128 {ktup(dst_slot)}, %[kb{s & 1}] offset:{slot_tile * TILE + kt * 4 * RB + 512 * (s >> 1)}"


def v_reads(f, slot_tile, dst_slot):
    ks, d = f // 4, f % 4
    off = slot_tile * TILE + 2 * ks * RB + 512 * d      # (the per-lane base carries the V ring)
    return [f"ds_read_b64_tr_b16 {vtup(dst_slot, h)}, %[vb{h}] offset:{off}" for h in (0, 1)]


def m_phase(dt, j_slot, pv=True, qk=True, prefetch=True):
    """PV(j) then QK^T(j+1); j_slot = j mod 4 (the ring slot of tile j).  On entry the first
    NVPRE V^T fragments of tile j are in flight or landed (read at the end of the previous M
    phase, in that order); ends with the next M phase's first NVPRE V^T reads (tile j+1)."""
    mnem = "v_mfma_f32_32x32x16_" + dt
    ks_slot = (j_slot + 1) % 4            # K(j+1)
    mf = []
    if pv:
        for f in range(16):
            ks, d = f // 4, f % 4
            mf.append((("V", f), f"{mnem} {otup(d)}, {vtup(f % VS)}, {ptup(ks)}, {otup(d)}"))
    if qk:
        for f in range(16):
            s, kt = f // 2, f % 2
            src = sv(kt) if s else "0"
            mf.append((("K", f), f"{mnem} {sv(kt)}, {ktup(f % KS)}, {qtup(s)}, {src}"))
    G = len(mf)
    first, last = {}, {}
    for g, (tag, _) in enumerate(mf):
        first.setdefault(tag, g)
        last[tag] = g
    reads = []                             # (gap, order, [texts], tag)
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
            reads.append((g, 0, [k_read(f, ks_slot, f % KS)], ("K", f)))
    if prefetch:                           # next M phase's first V^T fragments (tile j+1)
        for f in range(NVPRE):
            lo = (last[("V", 16 - VS + f)] + 2) if pv else 0
            g = max(lo, G - 2 * NVPRE + 2 * f)
            reads.append((min(g, G), 2 + f, v_reads(f, ks_slot, f), ("N", f)))
    # issue order and waits: the V^T fragments 0..NVPRE-1 of this tile were issued last in the
    # previous M phase (8 reads), oldest first
    issued = []
    last_idx = {}
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
        if g < 0 or g >= G:
            continue
        tag, text = mf[g]
        if tag in last_idx and last_idx[tag] >= waited:
            n = min(len(issued) - last_idx[tag] - 1, 15)
            out.append(f"s_waitcnt lgkmcnt({n})")
            waited = len(issued) - n
        out.append(text)
    return out


def dma(which, i, slot):
    base = (VREG if which == "V" else 0) + slot * TILE + i * 1024
    srd = SVR if which == "V" else SKR
    return [f"s_add_u32 m0, %[kdst], {base}", "s_nop 0",
            f"buffer_load_dwordx4 %[dma{i}], s[{srd}:{srd + 3}], 0 offen lds"]


def dma_pieces(slot):
    return [dma(w, i, slot) for w in ("K", "V") for i in (0, 1)]


def dma_advance():
    out = []
    for r in (SKR, SVR):
        out += [f"s_add_u32 s{r}, s{r}, %[kstep]", f"s_addc_u32 s{r + 1}, s{r + 1}, 0",
                f"s_sub_i32 s{r + 2}, s{r + 2}, %[kstep]", f"s_max_i32 s{r + 2}, s{r + 2}, 0"]
    return out


def dma_tile(slot):
    """this wave's 4 pieces of the next tile (slot), then both descriptors advance one tile"""
    return sum(dma_pieces(slot), []) + dma_advance()


def softmax(dt, pieces=()):
    """P = exp2(S c - m) for the 32 scores of this lane, tile row sum; DMA pieces spread in"""
    ops = []
    if PK:
        for i in range(16):                 # score pairs (2i, 2i+1)
            t0 = TMP + 2 * (i % 4)
            tp, t1 = f"v[{t0}:{t0 + 1}]", t0 + 1
            _, dword = value_info(2 * i + 1)
            st = [[f"v_pk_fma_f32 {tp}, v[{SBASE + 2 * i}:{SBASE + 2 * i + 1}], v[{CP}:{CP + 1}], v[{NMP}:{NMP + 1}]"],
                  [f"v_exp_f32 v{t0}, v{t0}", f"v_exp_f32 v{t1}, v{t1}"],
                  [f"v_pk_add_f32 v[{LT}:{LT + 1}], v[{LT}:{LT + 1}], {tp}",
                   f"v_cvt_pk_{dt}_f32 v{PBASE + dword}, v{t0}, v{t1}"]]
            for k, txt in enumerate(st):
                ops.append((2 * i + 2 * k, 2 * i, txt))
        span = 36
        pre = [f"v_mov_b32 v{LT}, 0", f"v_mov_b32 v{LT + 1}, 0"]
        post = ["s_nop 0", f"v_add_f32 v{LT}, v{LT}, v{LT + 1}"]
    else:
        for v in range(32):
            t = f"v{TMP + v % 8}"
            _, dword = value_info(v)
            st = [[f"v_fma_f32 {t}, v{SBASE + v}, %[c], v{NM}"], [f"v_exp_f32 {t}, {t}"],
                  [f"v_mov_b32 v{LT}, {t}" if v == 0 else f"v_add_f32 v{LT}, v{LT}, {t}"]]
            if v & 1:
                st[2].append(f"v_cvt_pk_{dt}_f32 v{PBASE + dword}, v{TMP + (v - 1) % 8}, {t}")
            for k, txt in enumerate(st):
                ops.append((v + 2 * k, v, txt))
        span = 36
        pre, post = [], ["s_nop 0"]
    for n, pc in enumerate(pieces):         # one piece every quarter of the softmax
        ops.append((2 + (n * span) // max(1, len(pieces)), -1, pc))
    out = list(pre)
    for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1])):
        out += txt
    return out + post + [f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}"]


def v_phase(dt, slot, full, dma=True, sm=True):
    """softmax(j+1) (full) beside the DMA of the tile in `slot`"""
    pieces = dma_pieces(slot) if dma else []
    out = []
    if full and sm:
        if DMAMIX:
            out += (pieces[0] if pieces else []) + ["s_nop 7", "s_nop 7"]   # MFMA results -> VALU
            out += softmax(dt, pieces[1:])
        else:
            out += sum(pieces, []) + ["s_nop 7", "s_nop 7", "s_nop 3"]
            out += softmax(dt)
        # the 4-wave kernel's per-step redo test (3 VALU/SALU + a not-taken branch)
        out += [f"v_cmp_lt_f32 vcc, %[thr], v{LT}", "s_nop 1", "s_cbranch_vccnz .Lredo_%="]
    else:
        out += sum(pieces, [])
    return out + (dma_advance() if dma else [])


def epilogue(dt):
    inv, L, t, lse, cls, pinf = (f"v{TMP + i}" for i in range(6))
    out = ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_nop 7", "s_nop 7", "s_nop 3",
           f"v_mov_b32 {pinf}, 0x7f800000",
           f"v_mov_b32 {t}, v{LRUN}", "s_nop 1", f"v_permlane32_swap_b32 v{LRUN}, {t}", "s_nop 1",
           f"v_add_f32 {L}, v{LRUN}, {t}", f"v_rcp_f32 {inv}, {L}", f"v_log_f32 {lse}, {L}",
           f"v_mov_b32 {cls}, 0x63", f"v_cmp_class_f32 vcc, {L}, {cls}",
           f"v_cndmask_b32_e64 {inv}, {inv}, 1.0, vcc", f"v_sub_f32 {lse}, {lse}, v{NM}",
           f"v_mul_f32 {lse}, 0x3f317218, {lse}", f"v_cndmask_b32 {lse}, {lse}, {pinf}, vcc",
           f"buffer_store_dword {lse}, %[loff], %[lsrd], 0 offen"]
    n = 0
    for d in range(4):
        for gp in (0, 2):
            vb = 0 if n % 2 == 0 else 16
            n += 1
            vals = [f"v{vb + k}" for k in range(8)]
            w0 = vb + 8
            src = [f"a{ABASE_O + 16 * d + 4 * gp + k}" for k in range(8)]
            out += [f"v_accvgpr_read_b32 {vals[k]}, {src[k]}" for k in range(8)]
            out += [f"v_mul_f32 {vals[k]}, {vals[k]}, {inv}" for k in range(8)]
            out += [f"v_cvt_pk_{dt}_f32 v{w0 + k}, {vals[2 * k]}, {vals[2 * k + 1]}" for k in range(4)]
            out += ["s_nop 1", f"v_permlane32_swap_b32 v{w0}, v{w0 + 2}",
                    f"v_permlane32_swap_b32 v{w0 + 1}, v{w0 + 3}", "s_nop 1",
                    f"buffer_store_dwordx4 v[{w0}:{w0 + 3}], %[ooff], %[osrd], 0 offen offset:{64 * d + 16 * gp}",
                    "s_nop 1"]
    return out


def item_program(dt, full):
    out = ["s_waitcnt lgkmcnt(0)",
           f"v_mov_b32 v{NM}, 0", f"v_mov_b32 v{LRUN}, {'0' if full else '1.0'}",
           f"v_mov_b32 v{CP}, %[c]", f"v_mov_b32 v{CP + 1}, %[c]",
           f"v_mov_b32 v{NMP}, 0", f"v_mov_b32 v{NMP + 1}, 0"]
    out += [f"buffer_load_dwordx4 {qtup(s)}, %[qoff], %[qsrd], 0 offen offset:{32 * s}" for s in range(8)]
    out += [f"v_accvgpr_write_b32 a{ABASE_O + i}, 0" for i in range(64)]
    # DMA descriptors at tile 0
    for r, lo, hi in ((SKR, "kblo", "kbhi"), (SVR, "vblo", "vbhi")):
        out += [f"s_mov_b32 s{r}, %[{lo}]", f"s_mov_b32 s{r + 1}, %[{hi}]",
                f"s_mov_b32 s{r + 2}, %[kvbytes]", f"s_mov_b32 s{r + 3}, 0x20000"]
    out += dma_tile(0) + dma_tile(1)
    out += ["s_waitcnt vmcnt(4)", "s_barrier"]          # Q and tile 0 landed, published
    if not full:
        # skeleton: P = the first Q fragments (random bf16 data for the PV MFMAs)
        out += ["s_waitcnt vmcnt(4)"]
        out += [f"v_accvgpr_read_b32 v{PBASE + i}, a{ABASE_Q + i}" for i in range(16)]
    def loop(group):
        uid = f"{group}_%="
        body, tail = [], []
        for ph in range(4):                          # ring phase: j mod 4
            body.append(f".Lph{ph}_{uid}:")
            if LAST:
                body += ["s_add_i32 s89, s88, 1", "s_cmp_ge_i32 s89, %[ntl]",
                         f"s_cbranch_scc1 .Llast{ph}_{uid}"]
                # the last step j = ntl - 1: PV only, no tile past the end
                tail.append(f".Llast{ph}_{uid}:")
                if group == "A":
                    tail += m_phase(dt, ph, qk=False, prefetch=False) + ["s_barrier"]
                    tail += ["s_waitcnt vmcnt(0)", "s_barrier"]
                else:
                    tail += v_phase(dt, (ph + 2) % 4, full, dma=False) + ["s_barrier"]
                    tail += m_phase(dt, ph, qk=False, prefetch=False) + ["s_waitcnt vmcnt(0)", "s_barrier"]
                tail.append(f"s_branch .Lexit_{uid}")
            if group == "A":
                body += m_phase(dt, ph) + ["s_barrier"]
                body += v_phase(dt, (ph + 3) % 4, full) + ["s_waitcnt vmcnt(4)", "s_barrier"]
            else:
                body += v_phase(dt, (ph + 2) % 4, full) + ["s_barrier"]
                body += m_phase(dt, ph) + ["s_waitcnt vmcnt(0)", "s_barrier"]
            body += ["s_add_i32 s88, s88, 1"]
            if not LAST:
                body += ["s_cmp_ge_i32 s88, %[ntl]", f"s_cbranch_scc1 .Lexit_{uid}"]
        body.append(f"s_branch .Lph0_{uid}")
        return body + tail

    # group A: M(-1) = QK(0), V(-1) = softmax(0) + DMA tile 2, then the loop
    prog_a = m_phase(dt, 3, pv=False) + ["s_barrier"]
    prog_a += v_phase(dt, 2, full) + ["s_waitcnt vmcnt(4)", "s_barrier", "s_mov_b32 s88, 0"]
    prog_a += loop("A") + [".Lexit_A_%=:"] + epilogue(dt) + ["s_branch .Lend_%="]
    # group B: an idle phase, M(-1), then the loop (V(j-1), M(j))
    prog_b = ["s_barrier"] + m_phase(dt, 3, pv=False) + ["s_waitcnt vmcnt(0)", "s_barrier",
                                                          "s_mov_b32 s88, 0"]
    prog_b += loop("B") + [".Lexit_B_%=:"] + epilogue(dt)
    out += ["s_cmp_eq_u32 %[grp], 0", "s_cbranch_scc0 .LgrpB_%="]
    out += prog_a + [".LgrpB_%=:"] + prog_b + [".Lend_%=:", "s_branch .Lfin_%="]
    if full:
        out += [".Lredo_%=:", "s_endpgm"]            # never taken (thr = inf in the probe)
    out += [".Lfin_%=:"]
    # M(-1): QK(0) reads K(0) from slot (3 + 1) % 4 = 0; its prefetch reads V(0) frags 0..3
    return out


SIG = ("const int kblo, const int kbhi, const int vblo, const int vbhi, const int kvbytes, "
       "const i32x4 qsrd, const i32x4 osrd, const i32x4 lsrd, const int kstep, const int kdst, "
       "const int ntl, const int grp, const float c, const float thr, const int kb0, const int kb1, "
       "const int vb0, const int vb1, const int dma0, const int dma1, const int qoff, "
       "const int ooff, const int loff")
OPS = ['[kblo] "s"(kblo)', '[kbhi] "s"(kbhi)', '[vblo] "s"(vblo)', '[vbhi] "s"(vbhi)',
       '[kvbytes] "s"(kvbytes)', '[qsrd] "s"(qsrd)', '[osrd] "s"(osrd)', '[lsrd] "s"(lsrd)',
       '[kstep] "s"(kstep)', '[kdst] "s"(kdst)', '[ntl] "s"(ntl)', '[grp] "s"(grp)',
       '[c] "s"(c)', '[thr] "s"(thr)',
       '[kb0] "v"(kb0)', '[kb1] "v"(kb1)', '[vb0] "v"(vb0)', '[vb1] "v"(vb1)',
       '[dma0] "v"(dma0)', '[dma1] "v"(dma1)', '[qoff] "v"(qoff)', '[ooff] "v"(ooff)',
       '[loff] "v"(loff)']


def clobbers():
    regs = [f'"v{i}"' for i in range(96)] + [f'"a{i}"' for i in range(128)]
    regs += [f'"s{i}"' for i in range(80, 96)]
    return ", ".join(regs + ['"vcc"', '"scc"', '"memory"'])


def emit(out=OUT):
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    lines = ["// GENERATED by tools/gen_pingpong.py (probe, not product code)", "#pragma once", "",
             "typedef __attribute__((ext_vector_type(4))) int i32x4;", ""]
    for full in (False, True):
        for dt in ("bf16",):
            prog = item_program(dt, full)
            name = f"pp_item_{'full' if full else 'skel'}_{dt}"
            lines.append(f"__device__ __forceinline__ void {name}({SIG}) {{")
            lines.append("    asm volatile(")
            lines += [f'        "{b}\\n"' for b in prog]
            lines.append("        :")
            lines.append("        : " + ",\n          ".join(OPS))
            lines.append(f"        : {clobbers()});")
            lines.append("}")
            lines.append("")
            print(name, len(prog), "lines")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--lead", type=int, default=LEAD)
    ap.add_argument("--no-pk", dest="pk", action="store_false")
    ap.add_argument("--no-dmamix", dest="dmamix", action="store_false")
    ap.add_argument("--no-last", dest="last", action="store_false")
    ap.add_argument("--out", default=OUT)
    a = ap.parse_args()
    LEAD, PK, DMAMIX, LAST = a.lead, a.pk, a.dmamix, a.last
    emit(a.out)

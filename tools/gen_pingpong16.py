"""Probe generator: the 8-wave ping-pong D = 128 forward of
tools/gen_pingpong.py with the bf16 MFMA shape v_mfma_f32_16x16x32 instead of 32x32x16, at the
same output tile per wave (32 query rows x 64 keys per step, O^T 128 x 32).

NOT part of the product.  It answers one question with a measurement (guide DVFS give-back item
7, cdna_hip_programming.md 5.4 rule 28): at the 1.4 kW board cap, does the chip hold a higher
clock on the 16x16x32 shape, enough to beat the 32x32x16 ping-pong per second?

Layout per wave (rows = the wave's 32 query rows as two 16-row tiles rt; g = lane >> 4):
  S^T(kt, rt) = K(kt) Q^T(rt)   16 keys x 16 rows, 4 k-steps of 32 d: lane = row 16 rt + (l & 15),
                                keys 16 kt + 4 g + r (r = 0..3)           32 MFMAs per tile
  O^T(dt, rt) += V^T(dt) P^T    16 d x 16 rows, 2 k-steps of 32 keys: k index m of lane group g
                                = key 32 ks + 16 (m >> 2) + 4 g + (m & 3), so P(ks, rt) is
                                cvt_pk of S^T(2 ks, rt) and S^T(2 ks + 1, rt) as they stand and
                                the V^T fragment is two ds_read_b64_tr_b16 blocks 16 keys apart
                                                                          32 MFMAs per tile
  row sums: per lane over its keys, reduced over the 4 lanes of a row (permlane32 / permlane16
  swaps) in the epilogue; K row reads ds_read_b128 at kv_off(16 kt + (l & 15), 4 s + g).

Register map per wave (256 = v[0:127] + a[0:127]):
  a[0:63] O^T (8 dt x 2 rt x 4), a[64:95] Q (2 rt x 4 s x 4), a[96:127] K fragment ring (8 x 4)
  v[0:31] S (4 kt x 2 rt x 4), v[32:47] P (2 ks x 2 rt x 4), v[48:55] scratch, v[56:59] tile row
  sums (rt 0 pair, rt 1 pair), v[60:61] (c, c), v[62:63] (-m, -m), v[64:95] V^T fragment ring,
  v[96:97] running row sums (rt 0, rt 1)

  python tools/gen_pingpong16.py     -> tools/probe/pingpong16_body.h
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "probe", "pingpong16_body.h")

HD = 128
RB = HD * 16           # one 8-row block of the kv_off image
TILE = 64 * HD * 2     # one K (or V) tile
VREG = 4 * TILE        # V ring after the 4 K slots
KS, VS = 8, 8          # fragment ring slots
LEAD = 6               # gaps an LDS read leads its MFMA
NVPRE = 4              # V^T fragments of the next M phase read at the end of this one
SBASE, PBASE, TMP = 0, 32, 48
LT, CP, NMP, LRUN = 56, 60, 62, 96   # LT: v[56:59] tile row sums (pairs per rt); LRUN: v[96:97]
PK = True              # softmax on packed fp32 (v_pk_fma_f32, v_pk_add_f32): half the fma / add
DMAMIX = True          # the VALU phase's 4 DMA pieces spread through the softmax
LAST = True            # the last step peeled: no QK^T / softmax of the tile past the end
ABASE_O, ABASE_Q, ABASE_K, VBASE_V = 0, 64, 96, 64
SKR, SVR = 80, 84      # DMA descriptors (next tile to load), K and V
SRA = 92


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
    b = SBASE + 4 * (2 * kt + rt)
    return f"v[{b}:{b + 3}]"


def ptup(ks, rt):
    b = PBASE + 4 * (2 * ks + rt)
    return f"v[{b}:{b + 3}]"


def k_read(f, slot_tile, dst_slot):
    s_, kt = f // 4, f % 4
    return f"ds_read_b128 {ktup(dst_slot)}, %[kb0] offset:{slot_tile * TILE + 4096 * kt + 512 * s_}"


def v_reads(f, slot_tile, dst_slot):
    ks, dt = f // 8, f % 8
    off = slot_tile * TILE + 8192 * ks + 512 * (dt >> 1)   # (the per-lane base carries the V ring)
    return [f"ds_read_b64_tr_b16 {vtup(dst_slot, h)}, %[vb{dt & 1}] offset:{off + 4096 * h}" for h in (0, 1)]


def m_phase(dt, j_slot, pv=True, qk=True, prefetch=True):
    """PV(j) then QK^T(j+1); j_slot = j mod 4 (the ring slot of tile j).  On entry the first
    NVPRE V^T fragments of tile j are in flight or landed (read at the end of the previous M
    phase, in that order); ends with the next M phase's first NVPRE V^T reads (tile j+1)."""
    mnem = "v_mfma_f32_16x16x32_" + dt
    ks_slot = (j_slot + 1) % 4            # K(j+1)
    mf = []
    if pv:
        for f in range(16):
            ks, d = f // 8, f % 8
            for rt in (0, 1):
                mf.append((("V", f), f"{mnem} {otup(d, rt)}, {vtup(f % VS)}, {ptup(ks, rt)}, {otup(d, rt)}"))
    if qk:
        for f in range(16):
            s_, kt = f // 4, f % 4
            for rt in (0, 1):
                src = sv(kt, rt) if s_ else "0"
                mf.append((("K", f), f"{mnem} {sv(kt, rt)}, {ktup(f % KS)}, {qtup(rt, s_)}, {src}"))
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
    """P = exp2(S c - m) for the 32 scores of this lane (2 rows x 16 keys), tile row sums per
    row (packed pairs); DMA pieces spread in"""
    ops = []
    for i in range(16):                 # score pairs v[2i:2i+1] = S(kt, rt) regs 2jj, 2jj+1
        kt, rt, jj = i // 4, (i // 2) % 2, i % 2
        dword = 4 * (2 * (kt // 2) + rt) + 2 * (kt % 2) + jj
        t0 = TMP + 2 * (i % 4)
        tp, t1 = f"v[{t0}:{t0 + 1}]", t0 + 1
        lt = f"v[{LT + 2 * rt}:{LT + 2 * rt + 1}]"
        st = [[f"v_pk_fma_f32 {tp}, v[{SBASE + 2 * i}:{SBASE + 2 * i + 1}], v[{CP}:{CP + 1}], v[{NMP}:{NMP + 1}]"],
              [f"v_exp_f32 v{t0}, v{t0}", f"v_exp_f32 v{t1}, v{t1}"],
              [f"v_pk_add_f32 {lt}, {lt}, {tp}",
               f"v_cvt_pk_{dt}_f32 v{PBASE + dword}, v{t0}, v{t1}"]]
        for k, txt in enumerate(st):
            ops.append((2 * i + 2 * k, 2 * i, txt))
    span = 36
    pre = [f"v_mov_b32 v{LT + k}, 0" for k in range(4)]
    post = ["s_nop 0", f"v_add_f32 v{LT}, v{LT}, v{LT + 1}", f"v_add_f32 v{LT + 2}, v{LT + 2}, v{LT + 3}"]
    for n, pc in enumerate(pieces):         # one piece every quarter of the softmax
        ops.append((2 + (n * span) // max(1, len(pieces)), -1, pc))
    out = list(pre)
    for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1])):
        out += txt
    return out + post + [f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}", f"v_add_f32 v{LRUN + 1}, v{LRUN + 1}, v{LT + 2}"]


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
        out += [f"v_max_f32 v{TMP}, v{LT}, v{LT + 2}", f"v_cmp_lt_f32 vcc, %[thr], v{TMP}", "s_nop 1",
                "s_cbranch_vccnz .Lredo_%="]
    else:
        out += sum(pieces, [])
    return out + (dma_advance() if dma else [])


def epilogue(dt):
    """row sums over the 4 lanes of each row, O / l -> bf16 (4 consecutive d per lane: 8-byte
    stores), LSE by the g = 0 lanes"""
    out = ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_nop 7", "s_nop 7", "s_nop 3"]
    inv = [f"v{TMP + 4}", f"v{TMP + 5}"]
    for rt in (0, 1):
        L, t, lse, cls, pinf = (f"v{TMP + i}" for i in range(5)) if rt == 0 else \
            (f"v{TMP + i}" for i in (0, 1, 2, 3, 6))
        out += [f"v_mov_b32 {pinf}, 0x7f800000",
                f"v_mov_b32 {t}, v{LRUN + rt}", "s_nop 1", f"v_permlane32_swap_b32 v{LRUN + rt}, {t}", "s_nop 1",
                f"v_add_f32 {L}, v{LRUN + rt}, {t}", f"v_mov_b32 {t}, {L}", "s_nop 1",
                f"v_permlane16_swap_b32 {L}, {t}", "s_nop 1", f"v_add_f32 {L}, {L}, {t}",
                f"v_rcp_f32 {inv[rt]}, {L}", f"v_log_f32 {lse}, {L}",
                f"v_mov_b32 {cls}, 0x63", f"v_cmp_class_f32 vcc, {L}, {cls}",
                f"v_cndmask_b32_e64 {inv[rt]}, {inv[rt]}, 1.0, vcc", f"v_sub_f32 {lse}, {lse}, v{NMP}",
                f"v_mul_f32 {lse}, 0x3f317218, {lse}", f"v_cndmask_b32 {lse}, {lse}, {pinf}, vcc",
                f"buffer_store_dword {lse}, %[loff{rt}], %[lsrd], 0 offen"]
    for d in range(8):
        for rt in (0, 1):
            vb = 0 if rt == 0 else 8
            vals = [f"v{vb + k}" for k in range(4)]
            src = [f"a{ABASE_O + 4 * (2 * d + rt) + k}" for k in range(4)]
            out += [f"v_accvgpr_read_b32 {vals[k]}, {src[k]}" for k in range(4)]
            out += [f"v_mul_f32 {vals[k]}, {vals[k]}, {inv[rt]}" for k in range(4)]
            out += [f"v_cvt_pk_{dt}_f32 v{vb + 4 + k}, {vals[2 * k]}, {vals[2 * k + 1]}" for k in range(2)]
            out += [f"buffer_store_dwordx2 v[{vb + 4}:{vb + 5}], %[ooff{rt}], %[osrd], 0 offen offset:{32 * d}"]
    return out


def item_program(dt, full):
    out = ["s_waitcnt lgkmcnt(0)",
           f"v_mov_b32 v{LRUN}, {'0' if full else '1.0'}", f"v_mov_b32 v{LRUN + 1}, {'0' if full else '1.0'}",
           f"v_mov_b32 v{CP}, %[c]", f"v_mov_b32 v{CP + 1}, %[c]",
           f"v_mov_b32 v{NMP}, 0", f"v_mov_b32 v{NMP + 1}, 0"]
    out += [f"buffer_load_dwordx4 {qtup(rt, s)}, %[qoff{rt}], %[qsrd], 0 offen offset:{64 * s}"
            for rt in (0, 1) for s in range(4)]
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
       "const int ntl, const int grp, const float c, const float thr, const int kb0, "
       "const int vb0, const int vb1, const int dma0, const int dma1, const int qoff0, const int qoff1, "
       "const int ooff0, const int ooff1, const int loff0, const int loff1")
OPS = ['[kblo] "s"(kblo)', '[kbhi] "s"(kbhi)', '[vblo] "s"(vblo)', '[vbhi] "s"(vbhi)',
       '[kvbytes] "s"(kvbytes)', '[qsrd] "s"(qsrd)', '[osrd] "s"(osrd)', '[lsrd] "s"(lsrd)',
       '[kstep] "s"(kstep)', '[kdst] "s"(kdst)', '[ntl] "s"(ntl)', '[grp] "s"(grp)',
       '[c] "s"(c)', '[thr] "s"(thr)',
       '[kb0] "v"(kb0)', '[vb0] "v"(vb0)', '[vb1] "v"(vb1)',
       '[dma0] "v"(dma0)', '[dma1] "v"(dma1)', '[qoff0] "v"(qoff0)', '[qoff1] "v"(qoff1)',
       '[ooff0] "v"(ooff0)', '[ooff1] "v"(ooff1)', '[loff0] "v"(loff0)', '[loff1] "v"(loff1)']


def clobbers():
    regs = [f'"v{i}"' for i in range(98)] + [f'"a{i}"' for i in range(128)]
    regs += [f'"s{i}"' for i in range(80, 96)]
    return ", ".join(regs + ['"vcc"', '"scc"', '"memory"'])


def emit(out=OUT):
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    lines = ["// GENERATED by tools/gen_pingpong16.py (probe, not product code)", "#pragma once", "",
             "typedef __attribute__((ext_vector_type(4))) int i32x4;", ""]
    for full in (False, True):
        for dt in ("bf16",):
            prog = item_program(dt, full)
            name = f"pp16_item_{'full' if full else 'skel'}_{dt}"
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

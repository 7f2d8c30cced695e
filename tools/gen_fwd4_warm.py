"""EXPERIMENT, not built: the warm-start / tail variant of tools/gen_fwd4.py.

Generate csrc/fmha_fwd4_body.h: the hand-scheduled body of the 4-wave D = 128 forward.

One workgroup = 4 waves, one per SIMD (the whole 512-register file per lane); a wave owns 64
query rows as two 32-row blocks rb.  The body of one work item (a 256-row query block of one
(batch, kv head)) is ONE asm statement with a fixed register map, generated here: hipcc's
register allocator cannot keep ~450 live registers in place across several large asm
statements (it splits and spills at every control-flow merge), so the whole key-tile pipeline,
its control flow, the rare rescale path and the epilogue live in one statement whose only
compiler-allocated operands are the item's scalars and per-lane offsets.

Step j of the key-tile loop runs, on one instruction stream,

  QK  S_{j+2}[rb][kt] = K_{j+2}[kt] . Q[rb]^T       32 x v_mfma_f32_32x32x16 (K frags from LDS)
  SM  P_{j+1} = exp2(S_{j+1} c - m), row sums       64 scores per lane: fma, exp, add, cvt
  PV  O[rb][dt] += V_j^T[dt] . P_j[rb]^T            32 x v_mfma_f32_32x32x16 (V^T by ds_read_tr)
  DMA K_{j+4}, V_{j+2} into 4-slot LDS rings         8 LDS-DMA pieces of 1 KiB per wave

with every instruction placed in an MFMA gap here (one v_exp per gap).  The loop is unrolled
over the 4 ring phases (slot offsets are immediates); per step a wave runs the unmasked body
(tile fully visible), the masked one (causal diagonal / window edge / ragged end) or an idle
one (past its last tile: DMA, barrier and prefetch only, so every wave meets every barrier).

Softmax without a row max in the loop: P = exp2(S c - m) against a reference m = the true max
of tile 0; after each step a lane's partial row sum of the new tile is compared with 2^slack;
if any passes, the rare path takes the tile's true max, rescales O and l and recomputes the
tile's P (nothing of that tile has reached O yet).  Results equal the online softmax of the
reference (softmax_hip.h:129-189) up to rounding.

Register map (per lane):
  a[0:127]    O^T accumulators, O[rb][dt] = a[64rb + 16dt : +15]
  a[128:191]  Q fragments (B operand of S^T), Q[rb][s] = a[128 + 32rb + 4s : +3]
  a[192:207]  K fragment ring, frag f in slot f % 4 (frags 0, 1 of the next step read early)
  a[240:255]  V^T fragment ring (4 slots)
  v[0:63]     S buffer A (4 accumulators rb*2 + kt);  v[64:127] S buffer B
  v[128:159]  P buffer A (8 x 4 dwords, rb*4 + ks);   v[160:191] P buffer B
  v[192:199]  score pipeline scratch;  v200-201 tile row sums;  v202-203 mask limits;
  v204-205    -m (log2 units) per rb;  v206-207 running row sums;  v208-215 misc
  s[80:87]    buffer descriptors of the step's DMA tiles (base advanced per tile, range clamped:
              the hardware range check ignores soffset, so tiles are addressed by the base)
  s[88:95]    step counter, DMA offsets, return address, compare masks
Even steps: S_{j+2} -> A, scores of j+1 in B, P_j in A, P_{j+1} -> B (odd steps swap).

The LDS image, fragment maps and P pair order are those of the 8-wave kernel
(fmha_fwd_kernel.h).

  python tools/gen_fwd4.py   (writes xf_flash_attention_cutlass_amd/csrc/fmha_fwd4_body.h)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc", "fmha_fwd4_body_warm.h")

HD = 128
RB = HD * 16          # bytes of one 8-row block of the kv_off image
TILE = 64 * HD * 2    # bytes of one K (or V) tile
VREG = 4 * TILE       # V ring after the K ring
QK_LEAD = 6           # QK MFMAs before the first PV MFMA (the step's V^T reads land meanwhile)
READ_LEAD = 5         # gaps between an LDS read and the MFMA that consumes it

# fixed registers
SBASE = (0, 64)       # S buffers A, B
PBASE = (128, 160)    # P buffers A, B
TMP = 192             # 8 scratch
LT, LIM, NM, LRUN = 200, 202, 204, 206
MISC = 208            # 208..215: 213 = +inf, 214 = -inf
PINF, NINF = 213, 214
ABASE_O, ABASE_Q, ABASE_K, ABASE_V = 0, 128, 192, 240
SJ, ST, SKO, SVO, SRA, SCM = 88, 89, 90, 91, 92, 94     # SRA: s[92:93], SCM: s[94:95]
STL = 96              # T - 2: the last step of the main loop + 1
SKR, SVR = 80, 84     # s[80:83] / s[84:87]: the K / V buffer descriptors of this step's DMA tiles

QK, SM, PV = 1, 2, 4

# schedule options (tools/gen_fwd4.py --variant N k=v ...; the default body uses these values):
#   dma_half  1: DMA issued in the first half of a step (K_{j+4}, V_{j+2});
#             2: in the second half, one tile further ahead (K_{j+5}, V_{j+3})
#   dma_free  1: no softmax instruction in a gap that carries a DMA piece
#   no_dma / no_barrier / no_sm: timing probes only (results wrong)
OPTS = dict(dma_half=1, dma_free=0, no_dma=0, no_barrier=0, no_sm=0)


def sv(buf, i):          # S accumulator tuple i (rb*2+kt) of buffer buf
    b = SBASE[buf] + 16 * i
    return f"v[{b}:{b + 15}]"


def se(buf, v):          # score element v (rb*32 + kt*16 + r)
    return f"v{SBASE[buf] + v}"


def ptup(buf, i):        # P tuple i (rb*4+ks)
    b = PBASE[buf] + 4 * i
    return f"v[{b}:{b + 3}]"


def pe(buf, d):          # P dword d (0..31)
    return f"v{PBASE[buf] + d}"


def otup(rb, dt):
    b = ABASE_O + 64 * rb + 16 * dt
    return f"a[{b}:{b + 15}]"


def qtup(rb, s):
    b = ABASE_Q + 32 * rb + 4 * s
    return f"a[{b}:{b + 3}]"


def ktup(slot):
    b = ABASE_K + 4 * slot
    return f"a[{b}:{b + 3}]"


def vtup(slot, half=None):
    b = ABASE_V + 4 * slot
    if half is None:
        return f"a[{b}:{b + 3}]"
    return f"a[{b + 2 * half}:{b + 2 * half + 1}]"


def value_info(v):
    """score v: rb, kt, r, key offset within the tile minus 4*hh, P dword index"""
    rb, kt, r = v // 32, (v // 16) % 2, v % 16
    off = 32 * kt + 8 * (r >> 2) + (r & 3)
    ks = 2 * kt + (r >> 3)
    dword = (rb * 4 + ks) * 4 + ((r & 7) >> 1)
    return rb, kt, r, off, dword


def mfma_order(kind):
    qk = [("QK", f // 2, f % 2, rb) for f in range(16) for rb in (0, 1)] if kind & QK else []
    pv = [("PV", f // 4, f % 4, rb) for f in range(16) for rb in (0, 1)] if kind & PV else []
    if qk and pv:
        seq = qk[:QK_LEAD]
        i, j = QK_LEAD, 0
        while i < len(qk):
            seq.append(pv[j]); j += 1
            seq.append(qk[i]); i += 1
        seq += pv[j:]
        return seq
    return qk + pv


def sm_value_ops(dt, v, src_buf, dst_buf, mask, nt):
    """the softmax ops of score v: [(stage, [texts])], stage 0 fma, 1 exp(+mask), 2 add, 3 cvt"""
    rb, kt, r, off, dword = value_info(v)
    t = f"v{TMP + v % nt}"
    ops = [(0, [f"v_fma_f32 {t}, {se(src_buf, v)}, %[c], v{NM + rb}"])]
    ex = [f"v_exp_f32 {t}, {t}"]
    if mask:
        ex += [f"v_cmp_lt_i32 vcc, {off}, v{LIM + rb}", f"v_cndmask_b32 {t}, 0, {t}, vcc"]
    ops.append((1, ex))
    if v % 32 == 0:
        ops.append((2, [f"v_mov_b32 v{LT + rb}, {t}"]))
    else:
        ops.append((2, [f"v_add_f32 v{LT + rb}, v{LT + rb}, {t}"]))
    if v & 1:
        tp = f"v{TMP + (v - 1) % nt}"
        ops.append((2, [f"v_cvt_pk_{dt}_f32 {pe(dst_buf, dword)}, {tp}, {t}"]))
    return ops


def step_body(dt, ph, kind, mask, tail=False, prefetch=(), fillers=(), midwait=8):
    """instructions of one step at ring phase ph (= j mod 4).
    tail: a step past the last QK (j >= T - 2): no K reads / DMA; V^T read through the runtime
          slot bases in the idle S buffer (the tail runs at any ring phase)
    prefetch: instruction units placed after the mid-point barrier (the next item's loads)
    fillers: single instructions spread one per gap (O zeroing in the first QK step)
    midwait: vmcnt at the mid-point barrier (None: no wait, no barrier)"""
    par = ph & 1
    sn_buf, sc_buf = (0, 1) if par == 0 else (1, 0)      # S_{j+2} -> sn, scores of j+1 in sc
    pc_buf, pn_buf = (0, 1) if par == 0 else (1, 0)      # P_j in pc, P_{j+1} -> pn
    kro = ((ph + 2) & 3) * TILE                          # K_{j+2}
    vro = (ph & 3) * TILE                                # V_j
    kno = ((ph + 3) & 3) * TILE                          # K_{j+3}: the next step's frags 0, 1
    if OPTS["dma_half"] == 1:
        kdo = (ph & 3) * TILE                            # K_{j+4} (DMA)
        vdo = VREG + ((ph + 2) & 3) * TILE               # V_{j+2} (DMA)
    else:
        kdo = ((ph + 1) & 3) * TILE                      # K_{j+5}
        vdo = VREG + ((ph + 3) & 3) * TILE               # V_{j+3}

    mf = mfma_order(kind)
    G = len(mf)
    mid = G // 2
    mfma = [None] * G
    need = [None] * G
    mnem = "v_mfma_f32_32x32x16_" + dt
    kfirst, klast, vfirst, vlast = {}, {}, {}, {}
    for g, (t, a, b, rb) in enumerate(mf):
        if t == "QK":
            s, kt = a, b
            f = 2 * s + kt
            acc = sv(sn_buf, rb * 2 + kt)
            src = "0" if s == 0 else acc
            mfma[g] = f"{mnem} {acc}, {ktup(f % 4)}, {qtup(rb, s)}, {src}"
            kfirst.setdefault(f, g); klast[f] = g
            need[g] = ("K", f)
        else:
            ks, d = a, b
            f = 4 * ks + d
            acc = otup(rb, d)
            mfma[g] = f"{mnem} {acc}, {vtup(f % 4)}, {ptup(pc_buf, rb * 4 + ks)}, {acc}"
            vfirst.setdefault(f, g); vlast[f] = g
            need[g] = ("V", f)

    reads = []   # (gap, order, text, tag)
    if kind & QK:
        for f in range(2, 16):
            s, kt = f // 2, f % 2
            lo = klast[f - 4] + 2 if f >= 4 else 0
            g = min(max(lo, kfirst[f] - READ_LEAD, 0), kfirst[f] - 1)
            reads.append((g, 0, f"ds_read_b128 {ktup(f % 4)}, %[kb{s & 1}] offset:{kro + kt * 4 * RB + 512 * (s >> 1)}", ("K", f)))
    if kind & PV:
        for f in range(16):
            ks, d = f // 4, f % 4
            lo = vlast[f - 4] + 2 if f >= 4 else 0
            g = min(max(lo, vfirst[f] - READ_LEAD, 0), vfirst[f] - 1)
            off = (0 if tail else vro) + 2 * ks * RB + 512 * d
            b0, b1 = (f"v{SBASE[sn_buf]}", f"v{SBASE[sn_buf] + 1}") if tail else ("%[vb0]", "%[vb1]")
            reads.append((g, 1, f"ds_read_b64_tr_b16 {vtup(f % 4, 0)}, {b0} offset:{off}", ("V", f)))
            reads.append((g, 2, f"ds_read_b64_tr_b16 {vtup(f % 4, 1)}, {b1} offset:{off}", ("V", f)))
    for f in ((0, 1) if not tail else ()):
        lo = max(mid + 1, (klast[12 + f] + 2) if (kind & QK) else 0)
        g = max(lo, G - 8 + 2 * f)
        reads.append((min(g, G), 3, f"ds_read_b128 {ktup(f)}, %[kb0] offset:{kno + f * 4 * RB}", ("N", f)))

    def dma(which, i):
        # LDS-DMA piece i: 8 rows x 8 chunks; M0 = its LDS address (lane l lands at +16 l)
        srd = f"s[{SKR}:{SKR + 3}]" if which == "K" else f"s[{SVR}:{SVR + 3}]"
        base = kdo if which == "K" else vdo
        if OPTS["no_dma"]:
            return ["s_nop 0", "s_nop 0"]
        return [f"s_add_u32 m0, %[kdst], {base + i * 1024}",
                f"buffer_load_dwordx4 %[dma{i}], {srd}, 0 offen lds"]
    bar = [] if OPTS["no_barrier"] else ["s_barrier"]

    dmas = [] if tail else [(w, i) for i in range(4) for w in ("K", "V")]
    dma_gap = {}
    if G:
        for n, wi in enumerate(dmas):
            if OPTS["dma_half"] == 1:
                g = min(1 + (n * max(1, mid - 2)) // len(dmas), mid - 1)
            else:
                g = min(mid + 1 + (n * max(1, G - mid - 3)) // len(dmas), G - 1)
            dma_gap.setdefault(g, []).append(wi)
    nt = 8 if (OPTS["dma_free"] or G not in (0, 64)) else 4
    sm = []      # (gap, seq, texts)
    if kind & SM and not OPTS["no_sm"]:
        if G and OPTS["dma_free"]:
            # softmax values only in gaps without a DMA piece (those carry the DMA's issue cost)
            avail = [g for g in range(G) if g not in dma_gap]
            avail += list(range(G, G + 3))
            n_av = len(avail) - 3
            for v in range(64):
                i = (v * n_av) // 64
                for stage, txt in sm_value_ops(dt, v, sc_buf, pn_buf, mask, nt):
                    sm.append((avail[i + stage], 4 * v + stage, txt))
        else:
            span = G if G else 64
            for v in range(64):
                tg = (v * span) // 64
                for stage, txt in sm_value_ops(dt, v, sc_buf, pn_buf, mask, nt):
                    sm.append((tg + stage, 4 * v + stage, txt))

    out = []
    if G == 0:
        if OPTS["dma_half"] == 2:
            out += ["s_waitcnt vmcnt(8)"] + bar
        for w, i in dmas:
            a, b = dma(w, i)
            out += [a, "s_nop 0", b]
        if OPTS["dma_half"] == 1:
            out += ["s_waitcnt vmcnt(8)"] + bar
        for _, _, txt in sorted(sm, key=lambda x: (x[0], x[1])):
            out += txt
        out += [r[2] for r in sorted(reads, key=lambda x: (x[0], x[1]))]
        return out

    assert len(fillers) <= G
    pf_gap = {}
    for n, unit in enumerate(prefetch):
        g = mid + 1 + (n * max(1, G - mid - 1)) // max(1, len(prefetch))
        pf_gap.setdefault(min(g, G - 1), []).extend(unit)
    issued = ["N0", "N1"]               # the previous step's prefetch of K frags 0, 1
    last_idx = {("K", 0): 0, ("K", 1): 1}
    waited = 0
    rby = {}
    for g, o, txt, tag in reads:
        rby.setdefault(g, []).append((o, txt, tag))
    smby = {}
    for g, seq, txt in sm:
        smby.setdefault(g, []).append((seq, txt))

    def issue_reads(g, body):
        for o, txt, tag in sorted(rby.get(g, []), key=lambda x: x[0]):
            body.append(txt)
            issued.append(tag)
            if tag[0] in "KV":
                last_idx[tag] = len(issued) - 1

    for g in range(-1, G + 3):
        body = []
        if g == -1:
            issue_reads(-1, body)
            out += body
            continue
        if g < G:
            nd = need[g]
            if nd in last_idx and last_idx[nd] >= waited:
                n = min(len(issued) - last_idx[nd] - 1, 15)
                body.append(f"s_waitcnt lgkmcnt({n})")
                waited = len(issued) - n
            body.append(mfma[g])
            if g == mid and midwait is not None:
                body += [f"s_waitcnt vmcnt({midwait})"] + bar
            if g < len(fillers):
                body += fillers[g]
            body += pf_gap.get(g, [])
        else:
            # past the last MFMA nothing separates a gap's v_exp from the next gap's use of its
            # result: a VALU reading a transcendental's result needs one wait state
            body.append("s_nop 0")
        dm = dma_gap.get(g, [])
        body += [dma(w, i)[0] for w, i in dm]
        for seq, txt in sorted(smby.get(g, []), key=lambda x: x[0]):
            body += txt
        body += [dma(w, i)[1] for w, i in dm]
        issue_reads(g, body)
        out += body
    return out


def step_prep():
    """per step: the buffer descriptors of K_{j+4} and V_{j+2} (V clamped at tile 0): base
    advanced to the tile, range = what is left of the workgroup's keys (>= 0)"""
    ka, va = (4, 2) if OPTS["dma_half"] == 1 else (5, 3)
    out = [f"s_add_i32 s{ST}, s{SJ}, {ka}", f"s_mul_i32 s{SKO}, s{ST}, %[kstep]",
           f"s_add_i32 s{ST}, s{SJ}, {va}", f"s_max_i32 s{ST}, s{ST}, 0",
           f"s_mul_i32 s{SVO}, s{ST}, %[kstep]"]
    for r, lo, hi, off in ((SKR, "kblo", "kbhi", SKO), (SVR, "vblo", "vbhi", SVO)):
        out += [f"s_add_u32 s{r}, %[{lo}], s{off}", f"s_addc_u32 s{r + 1}, %[{hi}], 0",
                f"s_sub_i32 s{r + 2}, %[kvbytes], s{off}", f"s_max_i32 s{r + 2}, s{r + 2}, 0",
                f"s_mov_b32 s{r + 3}, 0x20000"]
    return out


def lim_dec():
    return [f"v_add_u32 v{LIM}, -64, v{LIM}", f"v_add_u32 v{LIM + 1}, -64, v{LIM + 1}"]


def redo_block(dt, par, uid):
    """rare path for the scores in buffer (1 - par) (even steps: B): true max, rescale, redo"""
    sc_buf = 1 if par == 0 else 0
    pn_buf = 1 if par == 0 else 0
    out = [f".Lredo{par}_{uid}:", "s_nop 7", "s_nop 7", "s_nop 3"]
    mx, t2, alpha = f"v{MISC}", f"v{MISC + 1}", f"v{MISC + 2}"
    for rb in (0, 1):
        out.append(f"v_mov_b32 {mx}, v{NINF}")
        for vv in range(32):
            v = rb * 32 + vv
            _, _, _, off, _ = value_info(v)
            out += [f"v_cmp_lt_i32 vcc, {off}, v{LIM + rb}",
                    f"v_cndmask_b32 {t2}, v{NINF}, {se(sc_buf, v)}, vcc",
                    f"v_max_f32 {mx}, {mx}, {t2}"]
        # combine the row's two lane halves
        out += [f"v_mov_b32 {t2}, {mx}", "s_nop 1", f"v_permlane32_swap_b32 {mx}, {t2}",
                "s_nop 1",
                f"v_max_f32 {mx}, {mx}, {t2}",
                # m_new = max(m_ref, mx c), m_ref = -nm; alpha = exp2(m_ref - m_new)
                f"v_mul_f32 {t2}, %[c], {mx}",
                f"v_max_f32_e64 {t2}, {t2}, -v{NM + rb}",
                f"v_add_f32 {alpha}, v{NM + rb}, {t2}",
                f"v_exp_f32_e64 {alpha}, -{alpha}",
                f"v_mul_f32 v{NM + rb}, -1.0, {t2}",
                "s_nop 0",
                f"v_mul_f32 v{LRUN + rb}, v{LRUN + rb}, {alpha}"]
        for i in range(64):
            a = f"a{ABASE_O + 64 * rb + i}"
            t = f"v{TMP + i % 8}"
            out += [f"v_accvgpr_read_b32 {t}, {a}", f"v_mul_f32 {t}, {t}, {alpha}",
                    f"v_accvgpr_write_b32 {a}, {t}"]
        out.append("s_nop 1")
        # the tile's softmax again, masked, against the new reference
        ops = []
        for vv in range(32):
            v = rb * 32 + vv
            for stage, txt in sm_value_ops(dt, v, sc_buf, pn_buf, True, 8):
                ops.append((vv + stage, 4 * vv + stage, txt))
        for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1])):
            out += txt
    out += ["s_nop 3", f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]
    return out


def redo_check(par, uid, tag):
    """after a step with SM: any lane's tile sum past the threshold -> rare path; l += tile sums"""
    return [f"v_cmp_lt_f32 vcc, %[thr], v{LT}",
            f"v_cmp_lt_f32_e64 s[{SCM}:{SCM + 1}], %[thr], v{LT + 1}",
            f"s_or_b64 vcc, vcc, s[{SCM}:{SCM + 1}]",
            "s_nop 1",
            f"s_cbranch_vccz .Lnr{tag}_{uid}",
            f"s_getpc_b64 s[{SRA}:{SRA + 1}]",
            f".Lpc{tag}_{uid}:",
            f"s_add_u32 s{SRA}, s{SRA}, .Lnr{tag}_{uid} - .Lpc{tag}_{uid}",
            f"s_addc_u32 s{SRA + 1}, s{SRA + 1}, 0",
            f"s_branch .Lredo{par}_{uid}",
            f".Lnr{tag}_{uid}:",
            f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}",
            f"v_add_f32 v{LRUN + 1}, v{LRUN + 1}, v{LT + 1}"]


def prefetch_units():
    """the next item's K tiles 0, 1 (into ring slots 0, 1, as its warm start expects) and Q
    fragments: buffer descriptors, then 8 LDS-DMA pieces and 16 loads; a unit stays together"""
    units = [[f"s_mov_b32 s{SKR}, %[nkblo]", f"s_mov_b32 s{SKR + 1}, %[nkbhi]",
              f"s_mov_b32 s{SKR + 2}, %[nkvb]", f"s_mov_b32 s{SKR + 3}, 0x20000",
              f"s_add_u32 s{SVR}, %[nkblo], %[kstep]", f"s_addc_u32 s{SVR + 1}, %[nkbhi], 0",
              f"s_sub_i32 s{SVR + 2}, %[nkvb], %[kstep]", f"s_max_i32 s{SVR + 2}, s{SVR + 2}, 0",
              f"s_mov_b32 s{SVR + 3}, 0x20000"]]
    for t, r in ((0, SKR), (1, SVR)):
        for i in range(4):
            units.append([f"s_add_u32 m0, %[kdst], {t * TILE + i * 1024}", "s_nop 0",
                          f"buffer_load_dwordx4 %[dma{i}], s[{r}:{r + 3}], 0 offen lds"])
    for rb in (0, 1):
        for s in range(8):
            units.append([f"buffer_load_dwordx4 {qtup(rb, s)}, %[nqoff{rb}], %[nqsrd], 0 offen offset:{32 * s}"])
    return units


def tail_step(dt, par, kind, prefetch, uid, tag):
    """one tail step at runtime ring slot j & 3 (V^T bases in the idle S buffer), parity par:
    active waves run kind (SM masked); idle ones only meet the barrier; prefetch: the next
    item's loads after the step's barrier (all K slots are free once every wave is past the
    last QK step)"""
    units = prefetch_units() if prefetch else ()
    vt = SBASE[0 if par == 0 else 1]     # the V^T slot bases live in the idle S buffer (no QK)
    out = lim_dec() if kind & SM else []
    out += [f"s_and_b32 s{ST}, s{SJ}, 3", f"s_mul_i32 s{ST}, s{ST}, {TILE}",
            f"v_add_u32 v{vt}, s{ST}, %[vb0]", f"v_add_u32 v{vt + 1}, s{ST}, %[vb1]",
            f"s_cmp_gt_i32 s{SJ}, %[tw]", f"s_cbranch_scc1 .Lti{tag}_{uid}"]
    out += step_body(dt, par, kind, True, tail=True, prefetch=units,
                     midwait=0 if (prefetch or kind & SM) else None)
    if kind & SM:
        out += redo_check(par, uid, f"t{tag}")
    out += [f"s_branch .Ltn{tag}_{uid}", f".Lti{tag}_{uid}:"]
    if prefetch or kind & SM:
        out += ["s_waitcnt vmcnt(0)", "s_barrier"]
    for u in units:
        out += u
    out += [f".Ltn{tag}_{uid}:", f"s_add_i32 s{SJ}, s{SJ}, 1"]
    return out


def item_program(dt, uid="%="):
    out = ["s_waitcnt lgkmcnt(0)"]
    # constants, state
    out += [f"v_mov_b32 v{PINF}, 0x7f800000", f"v_mov_b32 v{NINF}, 0xff800000",
            f"v_mov_b32 v{NM}, 0", f"v_mov_b32 v{NM + 1}, 0",
            f"v_mov_b32 v{LRUN}, 0", f"v_mov_b32 v{LRUN + 1}, 0",
            f"v_mov_b32 v{LIM}, %[lim0]", f"v_mov_b32 v{LIM + 1}, %[lim1]"]
    assert OPTS["dma_half"] == 1
    # warm start: the previous item's tail already issued this item's Q fragments and K tiles
    # 0, 1 (ring slots 0, 1); they are older than that item's 18 epilogue stores
    out += [f"s_cmp_eq_u32 %[pre], 0", f"s_cbranch_scc1 .Lcold_{uid}",
            "s_waitcnt vmcnt(18)", "s_barrier",
            f"ds_read_b128 {ktup(0)}, %[kb0] offset:0",
            f"ds_read_b128 {ktup(1)}, %[kb0] offset:{4 * RB}",
            f"s_branch .Lqk0_{uid}",
            f".Lcold_{uid}:"]
    # cold start: Q fragments straight into their AGPRs, DMA-only steps j = -4, -3 (K_0, K_1)
    for rb in (0, 1):
        for s in range(8):
            out.append(f"buffer_load_dwordx4 {qtup(rb, s)}, %[qoff{rb}], %[qsrd], 0 offen offset:{32 * s}")
    for j in (-4, -3):
        out += [f"s_mov_b32 s{SJ}, {j}"] + step_prep() + step_body(dt, j % 4, 0, False)
    out += ["s_waitcnt vmcnt(0)", f".Lqk0_{uid}:"]
    # j = -2: QK(0), the O accumulators zeroed in its gaps (4 AGPR writes per gap)
    zero = [[f"v_accvgpr_write_b32 a{ABASE_O + 4 * g + i}, 0" for i in range(4)] for g in range(32)]
    out += [f"s_mov_b32 s{SJ}, -2"] + step_prep() + step_body(dt, 2, QK, False, fillers=zero,
                                                               midwait=63)
    # reference max of tile 0 (S in buffer A), masked in place
    out += ["s_nop 7", "s_nop 7", "s_nop 3"]
    mx, t2 = f"v{MISC}", f"v{MISC + 1}"
    for rb in (0, 1):
        out.append(f"v_mov_b32 {mx}, v{NINF}")
        for vv in range(32):
            v = rb * 32 + vv
            _, _, _, off, _ = value_info(v)
            out += [f"v_cmp_lt_i32 vcc, {off}, v{LIM + rb}",
                    f"v_cndmask_b32 {se(0, v)}, v{NINF}, {se(0, v)}, vcc",
                    f"v_max_f32 {mx}, {mx}, {se(0, v)}"]
        out += [f"v_mov_b32 {t2}, {mx}", "s_nop 1", f"v_permlane32_swap_b32 {mx}, {t2}",
                "s_nop 1",
                f"v_max_f32 {mx}, {mx}, {t2}",
                f"v_mul_f32_e64 {t2}, -%[c], {mx}",
                f"v_cmp_lg_f32 vcc, v{NINF}, {mx}",
                f"v_cndmask_b32 v{NM + rb}, 0, {t2}, vcc"]
    out += [f"s_mov_b32 s{SJ}, -1"] + step_prep() + step_body(dt, 3, QK | SM, False)
    out += [f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}", f"v_add_f32 v{LRUN + 1}, v{LRUN + 1}, v{LT + 1}"]
    # main loop over steps j = 0 .. ntl-1, unrolled over the 4 ring phases
    out += [f"s_sub_i32 s{STL}, %[ntl], 2",
            f"s_mov_b32 s{SJ}, 0", f"s_cmp_ge_i32 s{SJ}, s{STL}", f"s_cbranch_scc1 .Ltail_{uid}"]
    for ph in range(4):
        par = ph & 1
        out.append(f".Lph{ph}_{uid}:")
        out += step_prep() + lim_dec()
        out += [f"s_cmp_gt_i32 s{SJ}, %[tw]", f"s_cbranch_scc1 .Li{ph}_{uid}",
                f"s_add_i32 s{ST}, s{SJ}, 1", f"s_cmp_lt_i32 s{ST}, %[ew]",
                f"s_cbranch_scc0 .Lm{ph}_{uid}"]
        out += step_body(dt, ph, QK | SM | PV, False)
        out += redo_check(par, uid, f"u{ph}")
        out.append(f"s_branch .Lnx{ph}_{uid}")
        out.append(f".Lm{ph}_{uid}:")
        out += step_body(dt, ph, QK | SM | PV, True)
        out += redo_check(par, uid, f"m{ph}")
        out.append(f"s_branch .Lnx{ph}_{uid}")
        out.append(f".Li{ph}_{uid}:")
        out += step_body(dt, ph, 0, False)
        out.append(f".Lnx{ph}_{uid}:")
        out += [f"s_add_i32 s{SJ}, s{SJ}, 1", f"s_cmp_ge_i32 s{SJ}, s{STL}",
                f"s_cbranch_scc1 .Ltail_{uid}"]
    out.append(f"s_branch .Lph0_{uid}")
    # rare path bodies
    out += redo_block(dt, 0, uid) + redo_block(dt, 1, uid)
    # tail: j = T-2 (softmax of the last tile + PV, the next item's loads after its barrier)
    # and j = T-1 (PV of the last tile); T = 1: only the latter, carrying the loads
    out += [f".Ltail_{uid}:", f"s_cmp_lt_i32 %[ntl], 2", f"s_cbranch_scc1 .LtB1_{uid}",
            f"s_bitcmp1_b32 s{SJ}, 0", f"s_cbranch_scc1 .LtA1_{uid}"]
    for par in (0, 1):
        out.append(f".LtA{par}_{uid}:")
        out += tail_step(dt, par, SM | PV, True, uid, f"a{par}")
        out += tail_step(dt, 1 - par, PV, False, uid, f"b{par}")
        out.append(f"s_branch .Lexit_{uid}")
    out.append(f".LtB1_{uid}:")
    out += tail_step(dt, 0, PV, True, uid, "bt")
    # epilogue: every wave's LDS reads done (the next item's DMA may then reuse any slot);
    # normalise, O rows (16-byte stores after a permlane32 exchange), LSE
    out.append(f".Lexit_{uid}:")
    out += ["s_waitcnt lgkmcnt(0)", "s_barrier", "s_nop 7", "s_nop 7", "s_nop 3"]
    inv, L, t, lse = f"v{MISC}", f"v{MISC + 1}", f"v{MISC + 2}", f"v{MISC + 3}"
    n = 0
    for rb in (0, 1):
        out += [f"v_mov_b32 {t}, v{LRUN + rb}", "s_nop 1", f"v_permlane32_swap_b32 v{LRUN + rb}, {t}",
                "s_nop 1",
                f"v_add_f32 {L}, v{LRUN + rb}, {t}",
                f"v_rcp_f32 {inv}, {L}",
                f"v_log_f32 {lse}, {L}",
                f"v_mov_b32 v{MISC + 7}, 0x63",
                f"v_cmp_class_f32 vcc, {L}, v{MISC + 7}",
                f"v_cndmask_b32_e64 {inv}, {inv}, 1.0, vcc",
                f"v_sub_f32 {lse}, {lse}, v{NM + rb}",
                f"v_mul_f32 {lse}, 0x3f317218, {lse}",
                f"v_cndmask_b32 {lse}, {lse}, v{PINF}, vcc",
                f"buffer_store_dword {lse}, %[loff{rb}], %[lsrd], 0 offen"]
        for d in range(4):
            for gp in (0, 2):
                vb = 0 if n % 2 == 0 else 32          # two alternating register sets (S buffer A)
                n += 1
                vals = [f"v{vb + k}" for k in range(8)]
                w0 = vb + 16
                src = [f"a{ABASE_O + 64 * rb + 16 * d + 4 * gp + k}" for k in range(8)]
                out += [f"v_accvgpr_read_b32 {vals[k]}, {src[k]}" for k in range(8)]
                out += [f"v_mul_f32 {vals[k]}, {vals[k]}, {inv}" for k in range(8)]
                out += [f"v_cvt_pk_{dt}_f32 v{w0}, {vals[0]}, {vals[1]}",
                        f"v_cvt_pk_{dt}_f32 v{w0 + 1}, {vals[2]}, {vals[3]}",
                        f"v_cvt_pk_{dt}_f32 v{w0 + 2}, {vals[4]}, {vals[5]}",
                        f"v_cvt_pk_{dt}_f32 v{w0 + 3}, {vals[6]}, {vals[7]}",
                        "s_nop 1",
                        f"v_permlane32_swap_b32 v{w0}, v{w0 + 2}",
                        f"v_permlane32_swap_b32 v{w0 + 1}, v{w0 + 3}",
                        "s_nop 1",
                        f"buffer_store_dwordx4 v[{w0}:{w0 + 3}], %[ooff{rb}], %[osrd], 0 offen offset:{64 * d + 16 * gp}",
                        "s_nop 1"]
    return out


def clobbers():
    regs = [f'"v{i}"' for i in range(216)] + [f'"a{i}"' for i in range(256)]
    regs += [f'"s{i}"' for i in range(SKR, STL + 1)]
    return ", ".join(regs + ['"vcc"', '"scc"', '"memory"'])


SIG = ("const int kblo, const int kbhi, const int vblo, const int vbhi, const int kvbytes, "
       "const i32x4 qsrd, const i32x4 osrd, "
       "const i32x4 lsrd, const int kstep, const int kdst, const int ntl, "
       "const int tw, const int ew, const float c, const float thr, const int kb0, const int kb1, "
       "const int vb0, const int vb1, const int dma0, const int dma1, const int dma2, "
       "const int dma3, const int lim0, "
       "const int lim1, const int qoff0, const int qoff1, const int ooff0, const int ooff1, "
       "const int loff0, const int loff1, const int pre, const i32x4 nqsrd, const int nkblo, "
       "const int nkbhi, const int nkvb, const int nqoff0, const int nqoff1")
OPS = ['[kblo] "s"(kblo)', '[kbhi] "s"(kbhi)', '[vblo] "s"(vblo)', '[vbhi] "s"(vbhi)',
       '[kvbytes] "s"(kvbytes)', '[qsrd] "s"(qsrd)', '[osrd] "s"(osrd)',
       '[lsrd] "s"(lsrd)', '[kstep] "s"(kstep)', '[kdst] "s"(kdst)',
       '[ntl] "s"(ntl)', '[tw] "s"(tw)', '[ew] "s"(ew)', '[c] "s"(c)', '[thr] "s"(thr)',
       '[kb0] "v"(kb0)', '[kb1] "v"(kb1)', '[vb0] "v"(vb0)', '[vb1] "v"(vb1)',
       '[dma0] "v"(dma0)', '[dma1] "v"(dma1)', '[dma2] "v"(dma2)', '[dma3] "v"(dma3)',
       '[lim0] "v"(lim0)', '[lim1] "v"(lim1)',
       '[qoff0] "v"(qoff0)', '[qoff1] "v"(qoff1)', '[ooff0] "v"(ooff0)', '[ooff1] "v"(ooff1)',
       '[loff0] "v"(loff0)', '[loff1] "v"(loff1)', '[pre] "s"(pre)', '[nqsrd] "s"(nqsrd)',
       '[nkblo] "s"(nkblo)', '[nkbhi] "s"(nkbhi)', '[nkvb] "s"(nkvb)', '[nqoff0] "v"(nqoff0)',
       '[nqoff1] "v"(nqoff1)']


def emit(out_path=OUT):
    lines = [
        "// GENERATED by tools/gen_fwd4.py -- do not edit by hand.",
        "// The 4-wave D = 128 forward's item body (fmha_fwd4_kernel.h): one asm statement with a",
        "// fixed register map; see the generator's docstring for the map and the schedule.",
        "#pragma once",
        '#include "fmha_common.h"',
        "",
        "namespace xfa {",
        "typedef __attribute__((ext_vector_type(4))) int i32x4;",
        "",
    ]
    for dt in ("bf16", "f16"):
        prog = item_program(dt)
        lines.append(f"__device__ __forceinline__ void fwd4_item_{dt}({SIG}) {{")
        lines.append("    asm volatile(")
        for b in prog:
            lines.append(f'        "{b}\\n"')
        lines.append("        :")
        lines.append("        : " + ",\n          ".join(OPS))
        lines.append(f"        : {clobbers()});")
        lines.append("}")
        lines.append("")
        print(dt, len(prog), "instructions/labels")
    lines.append("}  // namespace xfa")
    open(out_path, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import sys
    args = sys.argv[1:]
    if args and args[0] == "--variant":
        n = int(args[1])
        for kv in args[2:]:
            k, v = kv.split("=")
            OPTS[k] = int(v)
        emit(OUT.replace(".h", f"_v{n}.h"))
    else:
        emit()

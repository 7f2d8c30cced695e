"""Generate csrc/fmha_fwd4_body.h: the hand-scheduled body of the 4-wave D = 128 forward.

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
  a[192:223]  K fragment ring, frag f in slot f % 8 (frags 0..3 of the next step read early)
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
OUT = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc", "fmha_fwd4_body.h")

HD = 128
RB = HD * 16          # bytes of one 8-row block of the kv_off image
TILE = 64 * HD * 2    # bytes of one K (or V) tile
VREG = 4 * TILE       # V ring after the K ring
QK_LEAD = 6           # QK MFMAs before the first PV MFMA (the step's V^T reads land meanwhile)
READ_LEAD = 8         # gaps between an LDS read and the MFMA that consumes it
KS, VS = 8, 4         # K / V^T fragment ring slots (AGPRs a[192:192+4KS], a[256-4VS:256])
NPRE, NVPRE = 4, 0    # K / V^T fragments of the next step read in this step's second half
# (round 4, same-box A/B: the 8-slot K ring read 8 gaps ahead with 4 fragments prefetched
#  across the step boundary +2..4 % over 4 slots / 5 gaps / 2; deeper V^T reads and the DMA
#  issued after the barrier did not add to it)
ABL = set()           # timing ablations (results INVALID): novm nobar nolgkm nodma nosm noredo mfma16
EPI_IDLE = True       # a wave's epilogue runs in its first idle step (causal diagonal; round 4,
                      # same box: C2 causal +2.6 %, bit-identical; no idle steps non-causal)
# The loop layout is fall-through (masked / idle steps and redo stubs out of line; round 4, same
# box: +0.9 % causal, +0.2 % non-causal, bit-identical).  Options measured and dropped (DESIGN.md
# 3.1b keeps one line each): DMA after the barrier one tile further ahead (-1 %), the DMA pieces
# in gaps 0..7 (-2.8 %), even/odd gap placement (noise), warm start (-1.8 % causal), non-temporal
# Q / O (-4 %), pre-scaled Q (+5 % but LSE 4.9e-3 off, over the 1e-3 gate).

# fixed registers
SBASE = (0, 64)       # S buffers A, B
PBASE = (128, 160)    # P buffers A, B
TMP = 192             # 8 scratch
LT, LIM, NM, LRUN = 200, 202, 204, 206
MISC = 208            # 208..215: 213 = +inf, 214 = -inf
PINF, NINF = 213, 214
NVFIX = 216           # fixed VGPRs v[0:NVFIX-1]
ABASE_O, ABASE_Q, ABASE_K, ABASE_V = 0, 128, 192, 240


GUARDS = []   # assembler checks of the return-address signs, emitted after the whole program


def addc_ret(reg, ret, pc, back):
    """high word of a return address s_getpc + (ret - pc): the carry plus the sign extension of
    the offset (-1 when the return point lies before the stub, 0 after).  An assembler guard,
    placed at the end of the asm statement (where both labels are defined), fails the build if
    the layout ever contradicts the sign assumed here (round 4's redo fault: a stub moved after
    its return point kept the high word 0)."""
    GUARDS.extend([f".if ({ret} - {pc}) {'>= 0' if back else '< 0'}", ".err", ".endif"])
    return [f"s_addc_u32 s{reg}, s{reg}, {-1 if back else 0}"]


SJ, ST, SKO, SVO, SRA, SCM = 88, 89, 90, 91, 92, 94     # SRA: s[92:93], SCM: s[94:95]
SKR, SVR = 80, 84     # s[80:83] / s[84:87]: the K / V buffer descriptors of this step's DMA tiles

QK, SM, PV = 1, 2, 4


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
    b = 256 - 4 * VS + 4 * slot
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
    z = 1
    ops = [(0, [f"v_fma_f32 {t}, {se(src_buf, v)}, %[c], v{NM + rb}"])]
    ex = [f"v_exp_f32 {t}, {t}"]
    if mask:
        ex += [f"v_cmp_lt_i32 vcc, {off}, v{LIM + rb}", f"v_cndmask_b32 {t}, 0, {t}, vcc"]
    ops.append((z, ex))
    if v % 32 == 0:
        ops.append((z + 1, [f"v_mov_b32 v{LT + rb}, {t}"]))
    else:
        ops.append((z + 1, [f"v_add_f32 v{LT + rb}, v{LT + rb}, {t}"]))
    if v & 1:
        tp = f"v{TMP + (v - 1) % nt}"
        ops.append((z + 1, [f"v_cvt_pk_{dt}_f32 {pe(dst_buf, dword)}, {tp}, {t}"]))
    return ops


def mfma16_pair(text, dt):
    """timing probe `--abl mfma16` (results INVALID): one v_mfma_f32_32x32x16 (32 cycles) as two
    v_mfma_f32_16x16x32 (16 cycles each) on the same A / B registers and the first 8 accumulator
    registers - the same FLOPs, MFMA-pipe cycles and operand traffic as the 16x16x32 form of the
    loop, with its issue hold (8 of every 16 cycles) and its clock behaviour on real data"""
    import re
    m = re.match(r"(\S+) ([va])\[(\d+):(\d+)\], (\S+), (\S+), (.+)$", text)
    _, rf, lo, _, a, b, c = m.groups()
    lo = int(lo)
    out = []
    for h in (0, 1):
        acc = f"{rf}[{lo + 4 * h}:{lo + 4 * h + 3}]"
        src = "0" if c == "0" else acc if c.startswith(rf + "[") else c
        out.append(f"v_mfma_f32_16x16x32_{dt} {acc}, {a}, {b}, {src}")
    return "\\n".join(out)


def step_body(dt, ph, kind, mask, vm=8):
    """instructions of one step at ring phase ph (= j mod 4)"""
    par = ph & 1
    sn_buf, sc_buf = (0, 1) if par == 0 else (1, 0)      # S_{j+2} -> sn, scores of j+1 in sc
    pc_buf, pn_buf = (0, 1) if par == 0 else (1, 0)      # P_j in pc, P_{j+1} -> pn
    kro = ((ph + 2) & 3) * TILE                          # K_{j+2}
    vro = (ph & 3) * TILE                                # V_j
    kno = ((ph + 3) & 3) * TILE                          # K_{j+3}: the next step's frags 0, 1
    kdo = ph % 4 * TILE                                  # K_{j+4} (DMA)
    vno = ((ph + 1) & 3) * TILE                          # V_{j+1}: the next step's first V^T frags
    vdo = VREG + (ph + 2) % 4 * TILE                     # V_{j+2} (DMA)

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
            src = acc if s else "0"
            mfma[g] = f"{mnem} {acc}, {ktup(f % KS)}, {qtup(rb, s)}, {src}"
            if "mfma16" in ABL:
                mfma[g] = mfma16_pair(mfma[g], dt)
            kfirst.setdefault(f, g); klast[f] = g
            need[g] = ("K", f)
        else:
            ks, d = a, b
            f = 4 * ks + d
            acc = otup(rb, d)
            mfma[g] = f"{mnem} {acc}, {vtup(f % VS)}, {ptup(pc_buf, rb * 4 + ks)}, {acc}"
            if "mfma16" in ABL:
                mfma[g] = mfma16_pair(mfma[g], dt)
            vfirst.setdefault(f, g); vlast[f] = g
            need[g] = ("V", f)

    reads = []   # (gap, order, text, tag)
    if kind & QK:
        for f in range(NPRE, 16):
            s, kt = f // 2, f % 2
            lo = klast[f - KS] + 2 if f >= KS else 0
            g = min(max(lo, kfirst[f] - READ_LEAD, 0), kfirst[f] - 1)
            reads.append((g, 0, f"ds_read_b128 {ktup(f % KS)}, %[kb{s & 1}] offset:{kro + kt * 4 * RB + 512 * (s >> 1)}", ("K", f)))
    if kind & PV:
        for f in range(NVPRE, 16):
            ks, d = f // 4, f % 4
            lo = vlast[f - VS] + 2 if f >= VS else 0
            g = min(max(lo, vfirst[f] - READ_LEAD, 0), vfirst[f] - 1)
            off = vro + 2 * ks * RB + 512 * d
            reads.append((g, 1, f"ds_read_b64_tr_b16 {vtup(f % VS, 0)}, %[vb0] offset:{off}", ("V", f)))
            reads.append((g, 2, f"ds_read_b64_tr_b16 {vtup(f % VS, 1)}, %[vb1] offset:{off}", ("V", f)))
    # the next step's first K (K_{j+3}) and V^T (V_{j+1}) fragments, both published at this
    # step's mid-point barrier, in one fixed order (the next step counts its waits on it)
    gprev = mid + 1
    for n, (w, f) in enumerate(prefetch_order()):
        if w == "N":
            lo = max(mid + 1, (klast[16 - KS + f] + 2) if (kind & QK) else 0)
            g = max(lo, G - 8 + 2 * f, gprev)
            s_, kt_ = f // 2, f % 2
            txt = [f"ds_read_b128 {ktup(f)}, %[kb{s_ & 1}] offset:{kno + kt_ * 4 * RB + 512 * (s_ >> 1)}"]
        else:
            lo = max(mid + 1, (vlast[16 - VS + f] + 2) if (kind & PV) else 0)
            g = max(lo, G - 8 + 2 * f, gprev)
            off = vno + 2 * (f // 4) * RB + 512 * (f % 4)
            txt = [f"ds_read_b64_tr_b16 {vtup(f, 0)}, %[vb0] offset:{off}",
                   f"ds_read_b64_tr_b16 {vtup(f, 1)}, %[vb1] offset:{off}"]
        gprev = g = min(g, G)
        for i, t in enumerate(txt):
            reads.append((g, 3 + 2 * n + i, t, (w, f)))

    def dma(which, i):
        # LDS-DMA piece i: 8 rows x 8 chunks; M0 = its LDS address (lane l lands at +16 l)
        srd = f"s[{SKR}:{SKR + 3}]" if which == "K" else f"s[{SVR}:{SVR + 3}]"
        base = kdo if which == "K" else vdo
        return [f"s_add_u32 m0, %[kdst], {base + i * 1024}",
                f"buffer_load_dwordx4 %[dma{i}], {srd}, 0 offen lds"]

    dmas = [] if "nodma" in ABL else [(w, i) for i in range(4) for w in ("K", "V")]
    nt = 4 if G in (0, 64) else 8
    sm = []      # (gap, seq, texts)
    if kind & SM and not ("nosm" in ABL and kind & PV):
        span = G if G else 64
        for v in range(64):
            tg = (v * span) // 64
            for stage, txt in sm_value_ops(dt, v, sc_buf, pn_buf, mask, nt):
                sm.append((tg + stage, 4 * v + stage, txt))

    out = []
    if G == 0:
        for w, i in dmas:
            a, b = dma(w, i)
            out += [a, "s_nop 0", b]
        out += [f"s_waitcnt vmcnt({vm})", "s_barrier"]
        for _, _, txt in sorted(sm, key=lambda x: (x[0], x[1])):
            out += txt
        out += [r[2] for r in sorted(reads, key=lambda x: (x[0], x[1]))]
        return out

    dma_gap = {}
    for n, wi in enumerate(dmas):
        g = min(1 + (n * max(1, mid - 2)) // len(dmas), mid - 1)
        dma_gap.setdefault(g, []).append(wi)
    # one piece per gap: a gap's M0 writes all precede its loads below
    assert all(len(v) == 1 for v in dma_gap.values()), "two LDS-DMA pieces in one gap"
    # the previous step's prefetch of this step's first K / V^T fragments, in issue order
    issued, last_idx = [], {}
    for w, f in prefetch_order():
        for _ in range(1 if w == "N" else 2):
            issued.append((w, f))
        last_idx[("K" if w == "N" else "V", f)] = len(issued) - 1
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
                if "nolgkm" not in ABL or not (kind & PV):
                    body.append(f"s_waitcnt lgkmcnt({n})")
                waited = len(issued) - n
            body.append(mfma[g])
            if g == mid:
                main = kind & PV
                body += [] if ("novm" in ABL and main) else [f"s_waitcnt vmcnt({vm})"]
                body += [] if ("nobar" in ABL and main) else ["s_barrier"]
        else:
            # past the last MFMA nothing separates a gap's v_exp from the next gap's use of its
            # result: a VALU reading a transcendental's result needs one wait state
            if not (smby.get(g) or dma_gap.get(g) or rby.get(g)):
                continue
            body.append("s_nop 0")
        dm = dma_gap.get(g, [])
        body += [dma(w, i)[0] for w, i in dm]
        for seq, txt in sorted(smby.get(g, []), key=lambda x: x[0]):
            body += txt
        body += [dma(w, i)[1] for w, i in dm]
        issue_reads(g, body)
        out += body
    return out


def prefetch_order():
    """the next step's fragments read at the end of a step: K frags 0..NPRE-1 ("N"), then V^T
    frags 0..NVPRE-1 ("W")"""
    return [("N", f) for f in range(NPRE)] + [("W", f) for f in range(NVPRE)]


def step_prep(incr=False):
    """per step: the buffer descriptors of K_{j+4} and V_{j+2} (V clamped at tile 0): base
    advanced to the tile, range = what is left of the workgroup's keys (>= 0).  incr (the main loop, where the previous step's descriptors are one tile behind):
    advance both by one tile, 8 SALU instead of 15"""
    if incr:
        out = []
        for r in (SKR, SVR):
            out += [f"s_add_u32 s{r}, s{r}, %[kstep]", f"s_addc_u32 s{r + 1}, s{r + 1}, 0",
                    f"s_sub_i32 s{r + 2}, s{r + 2}, %[kstep]", f"s_max_i32 s{r + 2}, s{r + 2}, 0"]
        return out
    kl, vl = 4, 2
    out = [f"s_add_i32 s{ST}, s{SJ}, {kl}", f"s_mul_i32 s{SKO}, s{ST}, %[kstep]",
           f"s_add_i32 s{ST}, s{SJ}, {vl}", f"s_max_i32 s{ST}, s{ST}, 0",
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


def prologue_dma(dt):
    """the DMA-only prologue steps, after the Q loads: K_0 published at step -3's barrier (and
    Q landed), K_1 / V_0 in flight for the next steps"""
    out = [f"s_mov_b32 s{SJ}, -4"] + step_prep() + step_body(dt, 0, 0, False)
    out += [f"s_mov_b32 s{SJ}, -3"] + step_prep() + step_body(dt, 1, 0, False)
    return out + ["s_waitcnt vmcnt(8)"]        # Q landed (older than j=-3's DMA)


def item_program(dt, uid="%="):
    out = ["s_waitcnt lgkmcnt(0)"]
    # constants, state
    out += [f"v_mov_b32 v{PINF}, 0x7f800000", f"v_mov_b32 v{NINF}, 0xff800000",
            f"v_mov_b32 v{NM}, 0", f"v_mov_b32 v{NM + 1}, 0",
            f"v_mov_b32 v{LRUN}, 0", f"v_mov_b32 v{LRUN + 1}, 0",
            f"v_mov_b32 v{LIM}, %[lim0]", f"v_mov_b32 v{LIM + 1}, %[lim1]"]
    # Q fragments straight into their AGPRs
    for rb in (0, 1):
        for s in range(8):
            out.append(f"buffer_load_dwordx4 {qtup(rb, s)}, %[qoff{rb}], %[qsrd], 0 offen offset:{32 * s}")
    # O accumulators zero (while Q and the first tiles are in flight)
    for i in range(128):
        out.append(f"v_accvgpr_write_b32 a{ABASE_O + i}, 0")
    # prologue steps j = -4, -3: DMA only (K_0, K_1); j = -2: QK(0); rowmax; j = -1: QK(1)+SM(0)
    out += prologue_dma(dt)
    out += [f"s_mov_b32 s{SJ}, -2"] + step_prep() + step_body(dt, 2, QK, False)
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
    out += main_loop_ff(dt, uid)
    # rare path bodies
    out += redo_block(dt, 0, uid) + redo_block(dt, 1, uid)
    out += epilogue(dt, uid)
    return out


def redo_check_ff(par, uid, tag):
    """redo_check with the common case falling through: a not-taken branch to an out-of-line stub
    (which sets the return address and enters the rare path) instead of a taken branch around the
    stub; returns (inline part, stub)"""
    inline = [f"v_cmp_lt_f32 vcc, %[thr], v{LT}",
              f"v_cmp_lt_f32_e64 s[{SCM}:{SCM + 1}], %[thr], v{LT + 1}",
              f"s_or_b64 vcc, vcc, s[{SCM}:{SCM + 1}]",
              "s_nop 1",
              f"s_cbranch_vccnz .Lrc{tag}_{uid}",
              f".Lnr{tag}_{uid}:",
              f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}",
              f"v_add_f32 v{LRUN + 1}, v{LRUN + 1}, v{LT + 1}"]
    # the return point lies BEFORE the stub: a negative offset, so the high word adds its sign
    # extension (-1) with the carry
    stub = [f".Lrc{tag}_{uid}:",
            f"s_getpc_b64 s[{SRA}:{SRA + 1}]",
            f".Lpc{tag}_{uid}:",
            f"s_add_u32 s{SRA}, s{SRA}, .Lnr{tag}_{uid} - .Lpc{tag}_{uid}",
            *addc_ret(SRA + 1, f".Lnr{tag}_{uid}", f".Lpc{tag}_{uid}", True),
            f"s_branch .Lredo{par}_{uid}"]
    return inline, stub


def main_loop_ff(dt, uid):
    """main loop, fall-through layout: per phase the unmasked step runs straight into the next
    phase (no taken branch on the common path); the masked and idle steps and the redo stubs live
    after the loop and branch back"""
    out = [f"s_mov_b32 s{SJ}, 0"]
    if EPI_IDLE:
        out.append(f"s_mov_b32 s{SKO}, 0")          # (SKO is the prologue's temp) rows not stored
    out += [f"s_cmp_ge_i32 s{SJ}, %[ntl]", f"s_cbranch_scc1 .Lexit_{uid}"]
    tail = []
    for ph in range(4):
        par = ph & 1
        out.append(f".Lph{ph}_{uid}:")
        out += step_prep(incr=True) + lim_dec()
        out += [f"s_cmp_gt_i32 s{SJ}, %[tw]", f"s_cbranch_scc1 .Li{ph}_{uid}",
                f"s_add_i32 s{ST}, s{SJ}, 1", f"s_cmp_lt_i32 s{ST}, %[ew]",
                f"s_cbranch_scc0 .Lm{ph}_{uid}"]
        out += step_body(dt, ph, QK | SM | PV, False)
        inl, stub = redo_check_ff(par, uid, f"u{ph}")
        out += inl
        tail += stub
        out.append(f".Lnx{ph}_{uid}:")
        out += [f"s_add_i32 s{SJ}, s{SJ}, 1", f"s_cmp_ge_i32 s{SJ}, %[ntl]",
                f"s_cbranch_scc1 .Lexit_{uid}"]
        # out of line: the masked and the idle step of this phase
        tail.append(f".Lm{ph}_{uid}:")
        tail += step_body(dt, ph, QK | SM | PV, True)
        inl, stub = redo_check_ff(par, uid, f"m{ph}")
        tail += inl + [f"s_branch .Lnx{ph}_{uid}"] + stub
        tail.append(f".Li{ph}_{uid}:")
        tail += step_body(dt, ph, 0, False)
        if EPI_IDLE:
            # first idle step (after its barrier): the rows' epilogue, once
            tail += [f"s_cmp_eq_u32 s{SKO}, 0", f"s_cbranch_scc0 .Lnx{ph}_{uid}",
                     f"s_mov_b32 s{SKO}, 1",
                     f"s_getpc_b64 s[{SRA}:{SRA + 1}]",
                     f".Lpe{ph}_{uid}:",
                     f"s_add_u32 s{SRA}, s{SRA}, .Lnx{ph}_{uid} - .Lpe{ph}_{uid}",
                     # (.Lnx lies before this stub: negative offset, high word + -1 + carry)
                     *addc_ret(SRA + 1, f".Lnx{ph}_{uid}", f".Lpe{ph}_{uid}", True),
                     f"s_branch .Lepi_{uid}"]
        else:
            tail.append(f"s_branch .Lnx{ph}_{uid}")
    out.append(f"s_branch .Lph0_{uid}")
    if EPI_IDLE:
        tail += epilogue_idle(dt, uid)
    return out + tail


def epilogue(dt, uid):
    # epilogue: normalise, O rows (16-byte stores after a permlane32 exchange), LSE
    out = [f".Lexit_{uid}:"]
    out += ["s_waitcnt vmcnt(0) lgkmcnt(0)"]
    if EPI_IDLE:
        # a wave that went idle before the last step has stored its rows already
        out += [f"s_cmp_eq_u32 s{SKO}, 1", f"s_cbranch_scc1 .Lend_{uid}"]
    out += ["s_nop 7", "s_nop 7", "s_nop 3"]
    out += epilogue_core(dt)
    if EPI_IDLE:
        out.append(f".Lend_{uid}:")
    return out


def epilogue_idle(dt, uid):
    """EPI_IDLE: the epilogue as a routine for the first idle step of a wave (its rows have no
    key tile left: O and the row sums are final), entered with the return address in SRA, so
    its row stores leave while the workgroup's last waves still compute and the item's tail
    holds only their stores"""
    return ([f".Lepi_{uid}:", "s_nop 7", "s_nop 7", "s_nop 3"] + epilogue_core(dt) +
            [f"s_setpc_b64 s[{SRA}:{SRA + 1}]"])


def epilogue_core(dt):
    out = []
    inv, L, t, lse = f"v{MISC}", f"v{MISC + 1}", f"v{MISC + 2}", f"v{MISC + 3}"
    cls, pinf = f"v{MISC + 7}", f"v{PINF}"
    oo, lo = ("%[ooff0]", "%[ooff1]"), ("%[loff0]", "%[loff1]")
    n = 0
    for rb in (0, 1):
        out += [f"v_mov_b32 {t}, v{LRUN + rb}", "s_nop 1", f"v_permlane32_swap_b32 v{LRUN + rb}, {t}",
                "s_nop 1",
                f"v_add_f32 {L}, v{LRUN + rb}, {t}",
                f"v_rcp_f32 {inv}, {L}",
                f"v_log_f32 {lse}, {L}",
                f"v_mov_b32 {cls}, 0x63",
                f"v_cmp_class_f32 vcc, {L}, {cls}",
                f"v_cndmask_b32_e64 {inv}, {inv}, 1.0, vcc",
                f"v_sub_f32 {lse}, {lse}, v{NM + rb}",
                f"v_mul_f32 {lse}, 0x3f317218, {lse}",
                f"v_cndmask_b32 {lse}, {lse}, {pinf}, vcc",
                f"buffer_store_dword {lse}, {lo[rb]}, %[lsrd], 0 offen"]
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
                        f"buffer_store_dwordx4 v[{w0}:{w0 + 3}], {oo[rb]}, %[osrd], 0 offen offset:{64 * d + 16 * gp}",
                        "s_nop 1"]
    return out


def clobbers():
    regs = [f'"v{i}"' for i in range(NVFIX)] + [f'"a{i}"' for i in range(256)]
    regs += [f'"s{i}"' for i in range(SKR, SCM + 2)]
    return ", ".join(regs + ['"vcc"', '"scc"', '"memory"'])


SIG = ("const int kblo, const int kbhi, const int vblo, const int vbhi, const int kvbytes, "
       "const i32x4 qsrd, const i32x4 osrd, "
       "const i32x4 lsrd, const int kstep, const int kdst, const int ntl, "
       "const int tw, const int ew, const float c, const float thr, const int kb0, const int kb1, "
       "const int vb0, const int vb1, const int dma0, const int dma1, const int dma2, "
       "const int dma3, const int lim0, "
       "const int lim1, const int qoff0, const int qoff1, const int ooff0, const int ooff1, "
       "const int loff0, const int loff1")
OPS = ['[kblo] "s"(kblo)', '[kbhi] "s"(kbhi)', '[vblo] "s"(vblo)', '[vbhi] "s"(vbhi)',
       '[kvbytes] "s"(kvbytes)', '[qsrd] "s"(qsrd)', '[osrd] "s"(osrd)',
       '[lsrd] "s"(lsrd)', '[kstep] "s"(kstep)', '[kdst] "s"(kdst)',
       '[ntl] "s"(ntl)', '[tw] "s"(tw)', '[ew] "s"(ew)', '[c] "s"(c)', '[thr] "s"(thr)',
       '[kb0] "v"(kb0)', '[kb1] "v"(kb1)', '[vb0] "v"(vb0)', '[vb1] "v"(vb1)',
       '[dma0] "v"(dma0)', '[dma1] "v"(dma1)', '[dma2] "v"(dma2)', '[dma3] "v"(dma3)',
       '[lim0] "v"(lim0)', '[lim1] "v"(lim1)',
       '[qoff0] "v"(qoff0)', '[qoff1] "v"(qoff1)', '[ooff0] "v"(ooff0)', '[ooff1] "v"(ooff1)',
       '[loff0] "v"(loff0)', '[loff1] "v"(loff1)']


def emit(out=OUT):
    assert 192 + 4 * KS <= 256 - 4 * VS and 16 % KS == 0 and 16 % VS == 0
    assert NPRE <= KS and NVPRE <= VS
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
        prog += GUARDS
        GUARDS.clear()
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
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", type=int, default=KS, help="K fragment ring slots")
    ap.add_argument("--vs", type=int, default=VS, help="V^T fragment ring slots")
    ap.add_argument("--lead", type=int, default=READ_LEAD, help="gaps an LDS read leads its MFMA")
    ap.add_argument("--npre", type=int, default=NPRE, help="next-step K frags read early")
    ap.add_argument("--nvpre", type=int, default=NVPRE, help="next-step V^T frags read early")
    ap.add_argument("--abl", default="", help="timing ablations, comma list (results invalid)")
    ap.add_argument("--no-epi-idle", dest="epi_idle", action="store_false",
                    help="epilogue after the loop only")
    ap.add_argument("--qklead", type=int, default=QK_LEAD, help="QK MFMAs before the first PV MFMA")
    ap.add_argument("--out", default=OUT)
    a = ap.parse_args()
    KS, VS, READ_LEAD, NPRE, NVPRE = a.ks, a.vs, a.lead, a.npre, a.nvpre
    ABL = set(x for x in a.abl.split(",") if x)
    QK_LEAD = a.qklead
    EPI_IDLE = a.epi_idle
    emit(a.out)

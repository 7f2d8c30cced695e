"""Generate csrc/fmha_fwd8_body.h: the hand-scheduled body of the 4-wave fp8 (e4m3fn) forward.

The fp8 analogue of tools/gen_fwd4.py (read its docstring first): one workgroup = 4 waves, one
per SIMD, each wave 64 query rows as two 32-row blocks rb; one work item (a 256-row query block
of one (batch, kv head)) is ONE asm statement with a fixed register map.  Both GEMMs run on the
block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (E8M0 scales 1.0: twice the bf16 rate, 64 cycles
per MFMA); the fp8 operand layouts are those of fmha_fwd_fp8_kernel.h (probed in
tools/probe_fp8.hip):

  QK  S^T[rb][kt] = sum_s K_{j+2}[kt][s] . Q[rb][s]^T   8 MFMAs, K frag (kt, s) = 32 bytes of key
                                                        row 32 kt + lane%32 at d = 64 s + 32 hh
  SM  P_{j+1} = e4m3(exp2(S c - m)), fp32 row sums       64 scores per lane
  PV  O^T[rb][dt] += V_j^T[dt] . P_j[rb]^T               8 MFMAs, V^T frag dt by 4 x
                                                        ds_read_b64_tr_b8 (32 keys of d column)
  DMA K_{j+4}, V_{j+2} into 4-slot LDS rings             4 LDS-DMA pieces of 1 KiB per wave

P leaves the S^T accumulator with keys 32 kt + 8 d + 4 hh + i (i = 0..3) in the lane half hh;
two v_cvt_pk_fp8_f32 pack them into P dword 4 kt + d, which is directly the B operand of PV with
its k index permuted: k slot (h, byte j) is key 32 (j >> 4) + 8 ((j >> 2) & 3) + 4 h + (j & 3).
The V^T reads apply the same permutation (a ds_read_b64_tr_b8 takes each of its 8 rows from
its own lane's address: read kb, row b is key 16 kb + 8 (b >> 2) + 4 h + (b & 3)), so P needs
no cross-lane regroup (round 3's kernel paid one v_permlane32_swap per dword pair).
Softmax as the bf16 body: no row max in the loop (P against tile 0's true max, a tile whose
partial row sum passes 2^slack takes the rare rescale path; slack <= 8 keeps P <= 256 < 448, the
e4m3 maximum), c = softmax_scale log2(e) q_scale k_scale, O scaled by v_scale / l at the end.

Register map (per lane):
  a[0:127]    O^T accumulators, O[rb][dt] = a[64 rb + 16 dt : +15]
  a[128:159]  Q fragments, Q[rb][s] = a[128 + 16 rb + 8 s : +7]
  a[160:223]  K fragment ring: 8 slots, frag f = 2 kt + s of a step of parity p in slot 4 p + f
              (a step's four fragments are read in the previous step's second half)
  a[224:255]  V^T fragment ring (4 slots, frag dt in slot dt)
  v[0:63]     S buffer A (rb * 2 + kt);  v[64:127] S buffer B
  v[128:143]  P buffer A (rb * 8 + dword);  v[144:159] P buffer B
  v[160:175]  score pipeline scratch;  v176-177 tile row sums;  v178-179 mask limits;
  v180-181    -m (log2 units) per rb;  v182-183 running row sums;  v184-191 misc
              (189 = 127: the E8M0 scale 1.0, 190 = +inf, 191 = -inf)
  s[80:95]    as gen_fwd4.py (K / V descriptors advanced per tile, step counter, ...)

  python tools/gen_fwd8.py   (writes xf_flash_attention_cutlass_amd/csrc/fmha_fwd8_body.h)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc", "fmha_fwd8_body.h")

TILE = 64 * 128       # bytes of one fp8 K (or V) tile
VREG = 4 * TILE       # V ring after the K ring (LDS)
QK_LEAD = 6           # QK MFMAs before the first PV MFMA (round 4, same box: 6 +1.1 % causal /
                      # +0.9 % non-causal over 2; 1, 3, 4, 7, 8 within noise or below)
READ_LEAD = 4         # gaps an LDS read leads the MFMA that consumes it (at least)
NWPRE = 4             # V^T frags of the next step read in this step's second half (all: LEAD2)

SBASE = (0, 64)
PBASE = (128, 144)
TMP, NTMP = 160, 16
LT, LIM, NM, LRUN = 176, 178, 180, 182
MISC = 184
SC127, PINF, NINF = 189, 190, 191
NVFIX = 192
ABASE_O, ABASE_Q, ABASE_K, ABASE_V = 0, 128, 160, 224
SJ, ST, SKO, SVO, SRA, SCM = 88, 89, 90, 91, 92, 94
SKR, SVR = 80, 84
NDMA = 4              # LDS-DMA wave-instructions per step (2 K + 2 V pieces)
LEAD2 = True          # DMA one more step ahead: step j issues K_{j+5}, V_{j+3} (the 4-slot rings
                      # allow it) and the mid-point wait keeps two steps' pieces in flight
ABL = set()           # timing ablations of the main-loop steps (results INVALID): nodma nosm nobar nolgkm
STAMPS = False        # diagnostic phase stamps (--stamps, XFA_FWD8_STAMPS; tools/fwd8_stamps.py)

QK, SM, PV = 1, 2, 4
MNEM = "v_mfma_scale_f32_32x32x64_f8f6f4"


GUARDS = []   # assembler checks of the return-address signs, emitted after the whole program

# phase classes of the stamps build: the cycles since the previous stamp go to the class named
ST_U, ST_W, ST_M, ST_I, ST_REDO, ST_PRO, ST_EPI, ST_TAIL = range(8)
ST_NAMES = ["unmasked run", "mid-step wait", "masked run", "idle step", "redo", "prologue",
            "epilogue", "exit drain"]


def st(k):
    """stamp (STAMPS builds only): s_memtime, the delta into lane k of %[acc].  Its
    lgkmcnt(0) also retires the LDS reads in flight, so read the build's SHARES, not its times."""
    if not STAMPS:
        return []
    return ["s_memtime s[96:97]", "s_waitcnt lgkmcnt(0)", "s_sub_u32 s99, s96, s98", "s_mov_b32 s98, s96",
            f"v_readlane_b32 s97, %[acc], {k}", "s_nop 3", "s_add_u32 s97, s97, s99", "s_nop 3",
            f"v_writelane_b32 %[acc], s97, {k}"]


def addc_ret(reg, ret, pc, back):
    """high word of a return address s_getpc + (ret - pc): the carry plus the sign extension of
    the offset (-1 when the return point lies before the stub, 0 after).  An assembler guard,
    placed at the end of the asm statement (where both labels are defined), fails the build if
    the layout ever contradicts the sign assumed here (round 4's redo fault: a stub moved after
    its return point kept the high word 0)."""
    GUARDS.extend([f".if ({ret} - {pc}) {'>= 0' if back else '< 0'}", ".err", ".endif"])
    return [f"s_addc_u32 s{reg}, s{reg}, {-1 if back else 0}"]


def sv(buf, i):
    b = SBASE[buf] + 16 * i
    return f"v[{b}:{b + 15}]"


def se(buf, v):            # score v = rb * 32 + kt * 16 + r
    return f"v{SBASE[buf] + v}"


def ptup(buf, rb):
    b = PBASE[buf] + 8 * rb
    return f"v[{b}:{b + 7}]"


def otup(rb, dt):
    b = ABASE_O + 64 * rb + 16 * dt
    return f"a[{b}:{b + 15}]"


def qtup(rb, s):
    b = ABASE_Q + 16 * rb + 8 * s
    return f"a[{b}:{b + 7}]"


def ktup(slot, half=None):
    b = ABASE_K + 8 * slot
    if half is None:
        return f"a[{b}:{b + 7}]"
    return f"a[{b + 4 * half}:{b + 4 * half + 3}]"


def vtup(slot, kb=None):
    b = ABASE_V + 8 * slot
    if kb is None:
        return f"a[{b}:{b + 7}]"
    return f"a[{b + 2 * kb}:{b + 2 * kb + 1}]"


def value_info(v):
    """score v: rb, kt, r, key offset within the tile minus 4 hh, P dword"""
    rb, kt, r = v // 32, (v // 16) % 2, v % 16
    off = 32 * kt + 8 * (r >> 2) + (r & 3)
    dword = rb * 8 + 4 * kt + (r >> 2)
    return rb, kt, r, off, dword


def mfma_order(kind):
    qk = [("QK", f, rb) for f in range(4) for rb in (0, 1)] if kind & QK else []
    pv = [("PV", dt, rb) for dt in range(4) for rb in (0, 1)] if kind & PV else []
    if qk and pv:
        seq = qk[:QK_LEAD]
        i, j = QK_LEAD, 0
        while i < len(qk):
            seq.append(pv[j]); j += 1
            seq.append(qk[i]); i += 1
        seq += pv[j:]
        return seq
    return qk + pv


def sm_value_ops(v, src_buf, dst_buf, mask, seq=False):
    """softmax ops of score v: [(stage, [texts])]; stage 0 fma, 1 exp (+mask), 2 add + cvt
    (seq: a plain sequence)"""
    rb, kt, r, off, dword = value_info(v)
    t = f"v{TMP + v % NTMP}"
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
        tp = f"v{TMP + (v - 1) % NTMP}"
        pd = f"v{PBASE[dst_buf] + dword}"
        sel = " op_sel:[0,0,1]" if (r & 3) == 3 else ""
        ops.append((2, [f"v_cvt_pk_fp8_f32 {pd}, {tp}, {t}{sel}"]))
    return ops


def prefetch_order():
    """the next step's fragments read at the end of a step: all four K frags ("N"), then V^T
    frags 0..NWPRE-1 ("W")"""
    return [("N", f) for f in range(4)] + [("W", dt) for dt in range(NWPRE)]


def step_body(ph, kind, mask, vm=None, stc=None):
    """instructions of one step at ring phase ph (= j mod 4); stc = (class of the first half,
    class of its mid-point wait) for the stamps build"""
    run_c, wait_c = stc if stc else (ST_PRO, ST_PRO)
    par = ph & 1
    sn_buf, sc_buf = (0, 1) if par == 0 else (1, 0)      # S_{j+2} -> sn, scores of j+1 in sc
    pc_buf, pn_buf = (0, 1) if par == 0 else (1, 0)      # P_j in pc, P_{j+1} -> pn
    kro = ((ph + 2) & 3) * TILE                          # K_{j+2} (read in the previous step)
    vro = (ph & 3) * TILE                                # V_j
    kno = ((ph + 3) & 3) * TILE                          # K_{j+3}: the next step's frags
    vno = ((ph + 1) & 3) * TILE                          # V_{j+1}: the next step's first frags
    if vm is None:
        vm = 2 * NDMA if LEAD2 else NDMA
    kdo = ((ph + (1 if LEAD2 else 0)) & 3) * TILE       # K_{j+4} (LEAD2: K_{j+5}) (DMA)
    vdo = VREG + ((ph + (3 if LEAD2 else 2)) & 3) * TILE  # V_{j+2} (LEAD2: V_{j+3}) (DMA)
    kslot = lambda f, p: 4 * (p & 1) + f                 # noqa: E731

    mf = mfma_order(kind)
    G = len(mf)
    mid = G // 2
    mfma, need = [None] * G, [None] * G
    vfirst, vlast = {}, {}
    klast = {}
    for g, (t, a, rb) in enumerate(mf):
        if t == "QK":
            f = a
            kt, s = f // 2, f % 2
            acc = sv(sn_buf, rb * 2 + kt)
            src = acc if s else "0"
            mfma[g] = (f"{MNEM} {acc}, {ktup(kslot(f, par))}, {qtup(rb, s)}, {src}, "
                       f"v{SC127}, v{SC127} op_sel_hi:[0,0,0]")
            need[g] = ("K", f)
            klast[f] = g
        else:
            dt = a
            acc = otup(rb, dt)
            mfma[g] = (f"{MNEM} {acc}, {vtup(dt)}, {ptup(pc_buf, rb)}, {acc}, "
                       f"v{SC127}, v{SC127} op_sel_hi:[0,0,0]")
            vfirst.setdefault(dt, g); vlast[dt] = g
            need[g] = ("V", dt)

    reads = []    # (gap, order, text, tag)
    if kind & PV:
        for dt in range(NWPRE, 4):
            g = min(max(vlast.get(dt - 4, -3) + 2 if dt >= 4 else 0, vfirst[dt] - READ_LEAD, 0),
                    vfirst[dt] - 1)
            for kb in range(4):
                reads.append((g, kb, f"ds_read_b64_tr_b8 {vtup(dt, kb)}, %[va{dt}] offset:{vro + kb * 2048}",
                              ("V", dt)))
    gprev = mid + 1
    npar = (par + 1) & 1
    for n, (w, f) in enumerate(prefetch_order()):
        if w == "N":
            # slot 4 npar + f held this step's frag f two steps ago: free since the last step
            kt, s = f // 2, f % 2
            g = max(mid + 1, gprev)
            txt = [f"ds_read_b128 {ktup(kslot(f, npar), u)}, %[ka{2 * s + u}] offset:{kno + kt * 32 * 128}"
                   for u in (0, 1)]
        else:
            lo = max(mid + 1, (vlast[f] + 2) if (kind & PV) else 0)
            g = max(lo, gprev)
            txt = [f"ds_read_b64_tr_b8 {vtup(f, kb)}, %[va{f}] offset:{vno + kb * 2048}"
                   for kb in range(4)]
        gprev = g = min(g, G)
        for i, t in enumerate(txt):
            reads.append((g, 10 + 4 * n + i, t, (w, f)))

    def dma(which, i):
        srd = f"s[{SKR}:{SKR + 3}]" if which == "K" else f"s[{SVR}:{SVR + 3}]"
        base = kdo if which == "K" else vdo
        op = f"%[dk{i}]" if which == "K" else f"%[dv{i}]"
        return [f"s_add_u32 m0, %[kdst], {base + i * 1024}",
                f"buffer_load_dwordx4 {op}, {srd}, 0 offen lds"]

    main = bool(kind & PV)                    # a main-loop step (ablations touch only those)
    dmas = [] if ("nodma" in ABL and main) else [(w, i) for i in range(2) for w in ("K", "V")]
    sm = []
    if kind & SM and not ("nosm" in ABL and main):
        span = G if G else 16
        for v in range(64):
            tg = (v * span) // 64
            for stage, txt in sm_value_ops(v, sc_buf, pn_buf, mask):
                sm.append((tg + stage, 8 * v + stage, txt))

    out = []
    if G == 0:
        for w, i in dmas:
            a, b = dma(w, i)
            out += [a, "s_nop 0", b]
        out += st(run_c) + [f"s_waitcnt vmcnt({vm})", "s_barrier"] + st(wait_c)
        for _, _, txt in sorted(sm, key=lambda x: (x[0], x[1])):
            out += txt
        out += [r[2] for r in sorted(reads, key=lambda x: (x[0], x[1]))]
        return out

    dma_gap = {}
    for n, wi in enumerate(dmas):
        g = min(1 + (n * max(1, mid - 2)) // len(dmas), mid - 1)
        dma_gap.setdefault(g, []).append(wi)
    issued, last_idx = [], {}
    for w, f in prefetch_order():
        for _ in range(2 if w == "N" else 4):
            issued.append((w, f))
        last_idx[("K" if w == "N" else "V", f)] = len(issued) - 1
    waited = 0
    rby, smby = {}, {}
    for g, o, txt, tag in reads:
        rby.setdefault(g, []).append((o, txt, tag))
    for g, seq, txt in sm:
        smby.setdefault(g, []).append((seq, txt))

    def issue_reads(g, body):
        for o, txt, tag in sorted(rby.get(g, []), key=lambda x: x[0]):
            body.append(txt)
            issued.append(tag)
            if tag[0] in "KV":
                last_idx[tag] = len(issued) - 1

    for g in range(-1, G + 6):
        body = []
        if g == -1:
            issue_reads(-1, body)
            out += body
            continue
        if g < G:
            nd = need[g]
            if nd in last_idx and last_idx[nd] >= waited:
                n = min(len(issued) - last_idx[nd] - 1, 15)
                if not ("nolgkm" in ABL and main):
                    body.append(f"s_waitcnt lgkmcnt({n})")
                waited = len(issued) - n
            body.append(mfma[g])
            if g == mid:
                body += [] if ("nobar" in ABL and main) else (
                    st(run_c) + [f"s_waitcnt vmcnt({vm})", "s_barrier"] + st(wait_c))
        else:
            if not (smby.get(g) or dma_gap.get(g) or rby.get(g)):
                continue
            body.append("s_nop 0")
        # a gap's DMA pieces: each load right behind its own M0 (the first pair straddles the
        # gap's softmax ops, later ones an s_nop for the SALU M0 write -> LDS-DMA hazard).  The
        # short (8-MFMA) prologue steps place two pieces in one gap: emitting both M0 writes
        # before both loads sent the first piece to the second's LDS address.
        dm = dma_gap.get(g, [])
        if dm:
            body.append(dma(*dm[0])[0])
        for seq, txt in sorted(smby.get(g, []), key=lambda x: x[0]):
            body += txt
        if dm:
            body.append(dma(*dm[0])[1])
            for w, i in dm[1:]:
                a, b = dma(w, i)
                body += [a, "s_nop 0", b]
        issue_reads(g, body)
        out += body
    return out


def step_prep(incr=False):
    """the K_{j+4} / V_{j+2} descriptors (V clamped at tile 0); incr: one tile on"""
    if incr:
        out = []
        for r in (SKR, SVR):
            out += [f"s_add_u32 s{r}, s{r}, %[kstep]", f"s_addc_u32 s{r + 1}, s{r + 1}, 0",
                    f"s_sub_i32 s{r + 2}, s{r + 2}, %[kstep]", f"s_max_i32 s{r + 2}, s{r + 2}, 0"]
        return out
    kl, vl = (5, 3) if LEAD2 else (4, 2)
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


def softmax_block(src_buf, dst_buf, lo_v, hi_v):
    """the masked softmax of scores [lo_v, hi_v) as a plain sequence (rare path)"""
    ops = []
    for v in range(lo_v, hi_v):
        for stage, txt in sm_value_ops(v, src_buf, dst_buf, True, seq=True):
            ops.append((v - lo_v + stage, 8 * v + stage, txt))
    out = []
    for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1])):
        out += txt
    return out


def redo_block(par, uid):
    """rare path for the scores in buffer (1 - par): true max, rescale O and l, redo the tile"""
    sc_buf = 1 if par == 0 else 0
    pn_buf = 1 if par == 0 else 0
    # (the step's last XDL writes of O / S: 40 wait states before VALU reads them)
    out = [f".Lredo{par}_{uid}:", "s_nop 7", "s_nop 7", "s_nop 7", "s_nop 7", "s_nop 7"]
    mx, t2, alpha = f"v{MISC}", f"v{MISC + 1}", f"v{MISC + 2}"
    for rb in (0, 1):
        out.append(f"v_mov_b32 {mx}, v{NINF}")
        for vv in range(32):
            v = rb * 32 + vv
            _, _, _, off, _ = value_info(v)
            out += [f"v_cmp_lt_i32 vcc, {off}, v{LIM + rb}",
                    f"v_cndmask_b32 {t2}, v{NINF}, {se(sc_buf, v)}, vcc",
                    f"v_max_f32 {mx}, {mx}, {t2}"]
        out += [f"v_mov_b32 {t2}, {mx}", "s_nop 1", f"v_permlane32_swap_b32 {mx}, {t2}",
                "s_nop 1",
                f"v_max_f32 {mx}, {mx}, {t2}",
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
        out += softmax_block(sc_buf, pn_buf, rb * 32, rb * 32 + 32)
        out.append("s_nop 1")
    out += ["s_nop 3"] + st(ST_REDO) + [f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]
    return out


def item_program(dt, uid="%="):
    out = (["s_memtime s[96:97]", "s_waitcnt lgkmcnt(0)", "s_mov_b32 s98, s96"] if STAMPS else [])
    out += ["s_waitcnt lgkmcnt(0)"]
    out += [f"v_mov_b32 v{PINF}, 0x7f800000", f"v_mov_b32 v{NINF}, 0xff800000",
            f"v_mov_b32 v{SC127}, 0x7f",
            f"v_mov_b32 v{NM}, 0", f"v_mov_b32 v{NM + 1}, 0",
            f"v_mov_b32 v{LRUN}, 0", f"v_mov_b32 v{LRUN + 1}, 0",
            f"v_mov_b32 v{LIM}, %[lim0]", f"v_mov_b32 v{LIM + 1}, %[lim1]"]
    # Q fragments: rb, s -> 2 x 16 bytes at d = 64 s + 32 hh (+ 16)
    for rb in (0, 1):
        for s in range(2):
            for u in range(2):
                b = ABASE_Q + 16 * rb + 8 * s + 4 * u
                out.append(f"buffer_load_dwordx4 a[{b}:{b + 3}], %[qoff{rb}], %[qsrd], 0 offen "
                           f"offset:{64 * s + 16 * u}")
    for i in range(128):
        out.append(f"v_accvgpr_write_b32 a{ABASE_O + i}, 0")
    # prologue: j = -4, -3 DMA only (K_0, K_1; the K_0 frags read at -3's end); j = -2 QK(0);
    # tile 0's row max; j = -1 QK(1) + SM(0); then the loop
    if LEAD2:
        # j = -5 .. -3 DMA only (K_0 .. K_2, V_0); Q and K_0 landed at -3's wait (vmcnt 8)
        out += [f"s_mov_b32 s{SJ}, -5"] + step_prep() + step_body(3, 0, False)
    out += [f"s_mov_b32 s{SJ}, -4"] + step_prep() + step_body(0, 0, False)
    out += [f"s_mov_b32 s{SJ}, -3"] + step_prep() + step_body(1, 0, False)
    out += [f"s_waitcnt vmcnt({2 * NDMA if LEAD2 else NDMA})"]   # Q landed (older than the DMA in flight)
    out += [f"s_mov_b32 s{SJ}, -2"] + step_prep() + step_body(2, QK, False)
    out += ["s_nop 7", "s_nop 7", "s_nop 7", "s_nop 7", "s_nop 3"]
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
    out += [f"s_mov_b32 s{SJ}, -1"] + step_prep() + step_body(3, QK | SM, False)
    out += [f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}", f"v_add_f32 v{LRUN + 1}, v{LRUN + 1}, v{LT + 1}"]
    out += main_loop(uid, dt)
    out += redo_block(0, uid) + redo_block(1, uid)
    out += epilogue(dt, uid)
    return out


def main_loop(uid, dt):
    """per phase the unmasked step falls through into the next phase; the masked and idle steps
    and the redo stubs live after the loop and branch back (gen_fwd4.py main_loop_ff)"""
    out = st(ST_PRO) + [f"s_mov_b32 s{SJ}, 0", f"s_mov_b32 s{SKO}, 0",      # SKO: rows stored (EPI_IDLE)
                        f"s_cmp_ge_i32 s{SJ}, %[ntl]", f"s_cbranch_scc1 .Lexit_{uid}"]
    tail = []
    for ph in range(4):
        par = ph & 1
        out.append(f".Lph{ph}_{uid}:")
        out += step_prep(incr=True) + lim_dec()
        out += [f"s_cmp_gt_i32 s{SJ}, %[tw]", f"s_cbranch_scc1 .Li{ph}_{uid}",
                f"s_add_i32 s{ST}, s{SJ}, 1", f"s_cmp_lt_i32 s{ST}, %[ew]",
                f"s_cbranch_scc0 .Lm{ph}_{uid}"]
        out += step_body(ph, QK | SM | PV, False, stc=(ST_U, ST_W))
        inl, stub = redo_check_ff(par, uid, f"u{ph}", ST_U)
        out += inl + st(ST_U)
        tail += stub
        out.append(f".Lnx{ph}_{uid}:")
        out += [f"s_add_i32 s{SJ}, s{SJ}, 1", f"s_cmp_ge_i32 s{SJ}, %[ntl]",
                f"s_cbranch_scc1 .Lexit_{uid}"]
        tail.append(f".Lm{ph}_{uid}:")
        tail += step_body(ph, QK | SM | PV, True, stc=(ST_M, ST_W))
        inl, stub = redo_check_ff(par, uid, f"m{ph}", ST_M)
        tail += inl + st(ST_M) + [f"s_branch .Lnx{ph}_{uid}"] + stub
        tail.append(f".Li{ph}_{uid}:")
        tail += step_body(ph, 0, False, stc=(ST_I, ST_I)) + st(ST_I)
        # first idle step (after its barrier): the rows' epilogue, once
        tail += [f"s_cmp_eq_u32 s{SKO}, 0", f"s_cbranch_scc0 .Lnx{ph}_{uid}",
                 f"s_mov_b32 s{SKO}, 1",
                 f"s_getpc_b64 s[{SRA}:{SRA + 1}]",
                 f".Lpe{ph}_{uid}:",
                 f"s_add_u32 s{SRA}, s{SRA}, .Lnx{ph}_{uid} - .Lpe{ph}_{uid}",
                 *addc_ret(SRA + 1, f".Lnx{ph}_{uid}", f".Lpe{ph}_{uid}", True),     # (.Lnx lies before: negative offset)
                 f"s_branch .Lepi_{uid}"]
    out.append(f"s_branch .Lph0_{uid}")
    return out + tail + epilogue_idle(uid, dt)


def redo_check_ff(par, uid, tag, stc=ST_U):
    """redo_check with the common case falling through (a not-taken branch to an out-of-line
    stub that sets the return address); returns (inline part, stub)"""
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
    stub = [f".Lrc{tag}_{uid}:"] + st(stc) + [
            f"s_getpc_b64 s[{SRA}:{SRA + 1}]",
            f".Lpc{tag}_{uid}:",
            f"s_add_u32 s{SRA}, s{SRA}, .Lnr{tag}_{uid} - .Lpc{tag}_{uid}",
            *addc_ret(SRA + 1, f".Lnr{tag}_{uid}", f".Lpc{tag}_{uid}", True),
            f"s_branch .Lredo{par}_{uid}"]
    return inline, stub


def epilogue(dt, uid):
    """O = v_scale O / l as 16-byte rows of the output dtype (permlane32 exchange), LSE; skipped
    by a wave that stored its rows in its first idle step (gen_fwd4.py EPI_IDLE)"""
    return ([f".Lexit_{uid}:", "s_waitcnt vmcnt(0) lgkmcnt(0)"] + st(ST_TAIL) +
            [f"s_cmp_eq_u32 s{SKO}, 1", f"s_cbranch_scc1 .Lend_{uid}",
             "s_nop 7", "s_nop 7", "s_nop 7", "s_nop 7", "s_nop 3"] + epilogue_core(dt) +
            [f".Lend_{uid}:"] + (["s_waitcnt vmcnt(0)"] + st(ST_EPI) if STAMPS else []))


def epilogue_idle(uid, dt):
    """the epilogue as a routine for a wave's first idle step (return address in SRA)"""
    return ([f".Lepi_{uid}:"] + st(ST_I) + ["s_nop 7", "s_nop 7", "s_nop 7", "s_nop 7", "s_nop 3"] +
            epilogue_core(dt) + st(ST_EPI) + [f"s_setpc_b64 s[{SRA}:{SRA + 1}]"])


def epilogue_core(dt):
    out = []
    inv, L, t, lse, cls = f"v{MISC}", f"v{MISC + 1}", f"v{MISC + 2}", f"v{MISC + 3}", f"v{MISC + 4}"
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
                f"v_mul_f32 {inv}, %[vsc], {inv}",
                f"v_sub_f32 {lse}, {lse}, v{NM + rb}",
                f"v_mul_f32 {lse}, 0x3f317218, {lse}",
                f"v_cndmask_b32 {lse}, {lse}, v{PINF}, vcc",
                f"buffer_store_dword {lse}, %[loff{rb}], %[lsrd], 0 offen"]
        for d in range(4):
            for gp in (0, 2):
                vb = 0 if n % 2 == 0 else 32
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
    regs = [f'"v{i}"' for i in range(NVFIX)] + [f'"a{i}"' for i in range(256)]
    regs += [f'"s{i}"' for i in range(SKR, SCM + 2)] + ([f'"s{i}"' for i in range(96, 100)] if STAMPS else [])
    return ", ".join(regs + ['"vcc"', '"scc"', '"memory"'])


SIG = ("const int kblo, const int kbhi, const int vblo, const int vbhi, const int kvbytes, "
       "const i32x4 qsrd, const i32x4 osrd, const i32x4 lsrd, const int kstep, const int kdst, "
       "const int ntl, const int tw, const int ew, const float c, const float thr, const float vsc, "
       "const int ka0, const int ka1, const int ka2, const int ka3, "
       "const int va0, const int va1, const int va2, const int va3, "
       "const int dk0, const int dk1, const int dv0, const int dv1, const int lim0, const int lim1, "
       "const int qoff0, const int qoff1, const int ooff0, const int ooff1, const int loff0, "
       "const int loff1")
SOPS = ["kblo", "kbhi", "vblo", "vbhi", "kvbytes", "qsrd", "osrd", "lsrd", "kstep", "kdst", "ntl",
        "tw", "ew", "c", "thr", "vsc"]
VOPS = ["ka0", "ka1", "ka2", "ka3", "va0", "va1", "va2", "va3", "dk0", "dk1", "dv0", "dv1",
        "lim0", "lim1", "qoff0", "qoff1", "ooff0", "ooff1", "loff0", "loff1"]


def emit(out=OUT):
    lines = [
        "// GENERATED by tools/gen_fwd8.py -- do not edit by hand.",
        "// The 4-wave fp8 forward's item body (fmha_fwd8w_kernel.h): one asm statement with a",
        "// fixed register map; see the generator's docstring for the map and the schedule.",
        "#pragma once",
        '#include "fmha_common.h"',
        "",
        *(["#define XFA_FWD8_STAMPS 1            // diagnostic build (--stamps)"] if STAMPS else []),
        "namespace xfa {",
        "typedef __attribute__((ext_vector_type(4))) int i32x4;",
        "",
    ]
    ops = [f'[{o}] "s"({o})' for o in SOPS] + [f'[{o}] "v"({o})' for o in VOPS]
    for dt in ("bf16", "f16"):
        prog = item_program(dt)
        prog += GUARDS
        GUARDS.clear()
        sig = SIG + (", unsigned& acc" if STAMPS else "")
        lines.append(f"__device__ __forceinline__ void fwd8_item_{dt}({sig}) {{")
        lines.append("    asm volatile(")
        for b in prog:
            lines.append(f'        "{b}\\n"')
        lines.append('        : [acc] "+v"(acc)' if STAMPS else "        :")
        lines.append("        : " + ",\n          ".join(ops))
        lines.append(f"        : {clobbers()});")
        lines.append("}")
        lines.append("")
        print(dt, len(prog), "instructions/labels")
    lines.append("}  // namespace xfa")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--abl", default="", help="timing ablations, comma list (results invalid)")
    ap.add_argument("--no-lead2", dest="lead2", action="store_false",
                    help="DMA two steps ahead only (3 V^T fragments prefetched)")
    ap.add_argument("--qklead", type=int, default=QK_LEAD, help="QK MFMAs before the first PV MFMA")
    ap.add_argument("--stamps", action="store_true", help="diagnostic phase stamps (XFA_FWD8_STAMPS)")
    ap.add_argument("--out", default=OUT)
    a = ap.parse_args()
    ABL = set(x for x in a.abl.split(",") if x)
    STAMPS = a.stamps
    QK_LEAD = a.qklead
    LEAD2 = a.lead2
    # LEAD2: V_{j+3} overwrites V_{j-1}'s slot in step j's first half, before its mid barrier, so
    # every V^T fragment of a tile must be read in the previous step (none after a barrier)
    NWPRE = 4 if LEAD2 else 3
    emit(a.out)

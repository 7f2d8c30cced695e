"""Generate csrc/fmha_fwdpp_body.h: the hand-scheduled body of the 8-wave "ping-pong" D = 128
forward (csrc/fmha_fwdpp_kernel.h).

Round 5's structure (probe: tools/gen_pingpong.py): one workgroup = 8 waves x
32 query rows = the 4-wave kernel's 256-row item, TWO waves per SIMD (waves w and w + 4), each
with 256 registers.  A wave's work alternates between two phases, each closed by an s_barrier:

  M(j)  the MFMA phase: PV(j) then QK^T(j+1)  (32 x v_mfma_f32_32x32x16, K / V^T fragments
        read from LDS in the gaps, the next PV's first V^T fragments read at its end)
  V(j)  the VALU phase: softmax(j+1) (fma, exp, row sum per score, cvt per pair) and the
        wave's share of the LDS-DMA of tile j+3 (4 pieces of 1 KiB: 8 rows of K and of V)

and group B (waves 4-7) runs one phase behind group A (waves 0-3): on every SIMD one wave
issues MFMAs while its partner issues VALU / DMA.  K / V tiles live in 4-slot LDS rings (the
kv_off image of the 4-wave kernel); tile t is published at the barrier that closes global phase
2t-1 (group A: s_waitcnt vmcnt(4) after its V phase, group B: vmcnt(0) after its M phase).
Measured (probe, C2 shape non-causal, two boxes): 12-13 % more work per clock than the 4-wave
kernel, 3-4 % more per second at the 1.4 kW board power cap.

Per wave and step j (the loop is unrolled over the 4 ring phases; slot offsets are immediates):
  unmasked  j+1 <= t_w, j+1 < e_w : M(j), V(j)
  masked    j+1 <= t_w, j+1 >= e_w: M(j), V(j) with the key-limit mask in the softmax
  last      j == t_w              : PV(j) only, then the wave's epilogue (O, LSE stores) in V(j)
  idle      j > t_w               : DMA and barriers only
(t_w: the wave's last key tile with a visible key, e_w: its first tile needing the edge mask).
Softmax without a row max in the loop (the 4-wave kernel's scheme): P = exp2(S c - m) against
m = the masked max of tile 0; a V phase whose partial row sums pass 2^slack takes the rare path
(true max, O and l rescaled, softmax redone).

FEATURES (round 6): softcap and ALiBi in an out-of-line pass over the tile's raw scores before
its softmax (feature_block; tile 0 before its max, the ALiBi max lifted by the row's best bias).
Causal ALiBi (feat bit 2) is the linear bias w key: w off per score, the tile base folded into NM
as a frame shift (SHIFT), the true -m kept in NMTRUE for the rare path, the row constant put
back into the LSE by the epilogue.
LEFTWIN: the key test is two-sided per lane, (off - LIML) <u wid; tiles before %[lw] take the
masked step; a row with no visible key in tile 0 starts from m = +inf, so its first visible key
sends the tile down the rare path, which takes the true max.  A step whose tile
j+1 lies before %[fw] (the wave's first tile with a visible key) is an idle step: tile 0's P of
such a wave is all zero and stays in the P registers until step fw - 1, whose PV adds nothing.

PAGED (fwdpp_pg_item_*): K / V in a paged cache.  A wave's DMA share of a tile (8 rows) lies in
one page (power-of-two page size >= 8), so each wave builds its own descriptors per tile:
pg_load at a V phase's start (the SMEM load of its next page id; nothing in a V phase waits on
lgkmcnt for LDS reads before pg_compute retires it), pg_compute at its end (base = pool + page
id x page stride + row in page x row bytes, range = its rows below the sequence length).

Register map (per lane, 256 = v[0:127] + a[0:127]):
  a[0:63]    O^T accumulators (4 d tiles x 16)
  a[64:95]   Q fragments (8 x 4), the B operand of S^T = K Q^T
  a[96:127]  K fragment ring (8 slots x 4)
  v[0:31]    S (2 x 16: keys 0-31, 32-63 of the tile for this lane's row)
  v[32:47]   P (4 x 4 packed pairs), the B operand of O^T += V^T P^T
  v[48:55]   softmax scratch (epilogue / redo temps)
  v56 tile row sum, v57 -m, v58 running row sum, v59 key limit, v60-63 redo / first-max temps
  v[64:95]   V^T fragment ring (8 slots x 4)
  v96 the left key limit (LEFTWIN, stepped with v59), v97 its compare temp
  s[80:87]   DMA descriptors (K, V) of the next tile to load; s88 step, s89 temp, s90 stored,
  s[92:93]   return address, s[94:95] compare mask

  python tools/gen_fwdpp.py        (writes xf_flash_attention_cutlass_amd/csrc/fmha_fwdpp_body.h)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc", "fmha_fwdpp_body.h")

HD = 128
RB = HD * 16           # one 8-row block of the kv_off image
TILE = 64 * HD * 2     # one K (or V) tile
KS, VS = 8, 8          # fragment ring slots
LEAD = 4               # gaps an LDS read leads its MFMA (round 5 A/B: 4 +0.7 % causal over 6)
NVPRE = 4              # V^T fragments of the next PV read at the end of an M phase
SBASE, PBASE, TMP = 0, 32, 48
LT, NM, LRUN, LIM, MISC = 56, 57, 58, 59, 60
ABASE_O, ABASE_Q, ABASE_K, VBASE_V = 0, 64, 96, 64
SKR, SVR = 80, 84
SJ, ST, SST, SRA, SCM = 88, 89, 90, 92, 94
ABL = set()            # timing ablations (results INVALID): nosm noredo nopro nopq nopkv; noepiwait (valid)
# (tools/gen_fwd8pp.py reuses this generator's phase program for the fp8 kernel: it rebinds the
#  operand-specific functions below and these parameters)
XDL_NOPS = ["s_nop 7", "s_nop 7", "s_nop 3"]   # last MFMA write -> VALU read of O / S
VPH_NOPS = ["s_nop 7", "s_nop 7"]              # (a V phase: after its first DMA piece)
NPIECE = 4             # LDS-DMA pieces per wave per tile (A's publish wait keeps them in flight)
EPI_SCALE = None       # an SGPR operand O is also scaled by in the epilogue (fp8: %[vsc])
DMAMIX = True          # the V phase's DMA pieces 2-4 spread through the softmax (else all first)
PRO_V0 = False         # (experiment) the prologue's wait leaves tile 0's V pieces in flight
STAMPS = False         # diagnostic build: s_memtime per phase boundary, summed per class in lanes
                       # 0-7 of %[acc] (fmha_fwdpp_kernel.h XFA_FWDPP_STAMPS; read its SHARES only)
RING = 4               # K / V tile slots in LDS
DLEAD = 3              # V(j) loads tile j + DLEAD (needs RING > DLEAD: B's last read of tile t
                       # is in global phase 2t+3, A's load of tile t+RING in 2(t+RING-DLEAD)+3)

GUARDS = []            # assembler checks of the return-address signs, after the whole program
FEATURES = True        # the score features (softcap, ALiBi) behind %[feat] bits, as an out-of-line
                       # pass over S before each softmax (gen_fwd8pp / gen_fwdpp16 turn it off)
LEFTWIN = True         # two-sided key window in the masked steps (left windows: keys
                       # [LIML, LIML + %[wid]) of the tile, relative to this lane's offset 0)
LIML, TW = 96, 97      # the lane's left key limit (stepped -64 per tile); a compare temp
PAGED = False          # emitting the paged-K/V body (fwdpp_pg_item_*): per-wave page descriptors
SKEY, SPG, ST2 = 91, 94, 95   # (paged) this wave's next key row to set up, its page id, a temp
SHIFT, NMTRUE = 98, 99  # (causal ALiBi, feat bit 2) this tile's frame shift c w key0, the true -m


def addc_ret(reg, ret, pc, back):
    """high word of a return address s_getpc + (ret - pc) (see gen_fwd4.addc_ret)"""
    GUARDS.extend([f".if ({ret} - {pc}) {'>= 0' if back else '< 0'}", ".err", ".endif"])
    return [f"s_addc_u32 s{reg}, s{reg}, {-1 if back else 0}"]


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
    """score v (kt*16 + r) of this lane: key offset in the tile minus 4*hh, P dword"""
    kt, r = v // 16, v % 16
    off = 32 * kt + 8 * (r >> 2) + (r & 3)
    ks = 2 * kt + (r >> 3)
    return off, ks * 4 + ((r & 7) >> 1)


def k_read(f, slot_tile, dst_slot):
    s, kt = f // 2, f % 2
    return f"ds_read_b128 {ktup(dst_slot)}, %[kb{s & 1}] offset:{slot_tile * TILE + kt * 4 * RB + 512 * (s >> 1)}"


def v_reads(f, slot_tile, dst_slot):
    ks, d = f // 4, f % 4
    off = slot_tile * TILE + 2 * ks * RB + 512 * d          # (the lane base carries the V ring)
    return [f"ds_read_b64_tr_b16 {vtup(dst_slot, h)}, %[vb{h}] offset:{off}" for h in (0, 1)]


def m_phase(dt, j_slot, pv=True, qk=True):
    """PV(j) then QK^T(j+1) (j_slot = j mod 4); with qk the next PV's first NVPRE V^T fragments
    (tile j+1) are read at the end.  On entry with pv, this tile's first NVPRE V^T fragments are
    the only LDS reads in flight (the previous M phase's prefetch)."""
    mnem = "v_mfma_f32_32x32x16_" + dt
    nx = (j_slot + 1) % RING
    mf = []
    if pv:
        for f in range(16):
            ks, d = f // 4, f % 4
            mf.append((("V", f), f"{mnem} {otup(d)}, {vtup(f % VS)}, {ptup(ks)}, {otup(d)}"))
    if qk:
        for f in range(16):
            s, kt = f // 2, f % 2
            mf.append((("K", f), f"{mnem} {sv(kt)}, {ktup(f % KS)}, {qtup(s)}, {sv(kt) if s else '0'}"))
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
            g = max(lo, G - 2 * NVPRE + 2 * f)
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


def dma_pieces(slot):
    out = []
    for w, srd, base in (("K", SKR, 0), ("V", SVR, RING * TILE)):
        for i in (0, 1):
            out.append([f"s_add_u32 m0, %[kdst], {base + slot * TILE + i * 1024}", "s_nop 0",
                        f"buffer_load_dwordx4 %[dma{i}], s[{srd}:{srd + 3}], 0 offen lds"])
    return out


def pg_load():
    """(paged) issue the page-id load of the tile whose descriptors pg_compute sets up next: this
    wave's 8 rows from key SKEY (clamped to the last key, so the load stays in the sequence's
    block-table row); an SMEM load, so it is issued at a V phase's start and waited for at its end
    (no LDS read waits on lgkmcnt in between)"""
    return [f"s_add_i32 s{ST}, %[skv], -1", f"s_min_i32 s{ST}, s{SKEY}, s{ST}",
            f"s_lshr_b32 s{ST}, s{ST}, %[lgp]", f"s_lshl_b32 s{ST}, s{ST}, 2",
            f"s_load_dword s{SPG}, %[btab], s{ST}"]


def pg_compute():
    """(paged) the K / V descriptors of this wave's 8 rows from key SKEY: base = pool + page id x
    page stride + row in page x row bytes, range = its rows below the sequence length (rows past
    it read zeros); then SKEY += 64"""
    return ["s_waitcnt lgkmcnt(0)",
            f"s_and_b32 s{ST}, s{SKEY}, %[pmask]", f"s_mul_i32 s{ST}, s{ST}, %[rowb]",
            f"s_mul_hi_u32 s{ST2}, s{SPG}, %[pstr]", f"s_mul_i32 s{SPG}, s{SPG}, %[pstr]",
            f"s_add_u32 s{SPG}, s{SPG}, s{ST}", f"s_addc_u32 s{ST2}, s{ST2}, 0",
            f"s_add_u32 s{SKR}, %[kblo], s{SPG}", f"s_addc_u32 s{SKR + 1}, %[kbhi], s{ST2}",
            f"s_and_b32 s{SKR + 1}, s{SKR + 1}, 0xffff",
            f"s_add_u32 s{SVR}, %[vblo], s{SPG}", f"s_addc_u32 s{SVR + 1}, %[vbhi], s{ST2}",
            f"s_and_b32 s{SVR + 1}, s{SVR + 1}, 0xffff",
            f"s_sub_i32 s{ST}, %[skv], s{SKEY}", f"s_max_i32 s{ST}, s{ST}, 0", f"s_min_i32 s{ST}, s{ST}, 8",
            f"s_mul_i32 s{SKR + 2}, s{ST}, %[rowb]", f"s_mov_b32 s{SVR + 2}, s{SKR + 2}",
            f"s_add_u32 s{SKEY}, s{SKEY}, 64"]


def dma_advance():
    if PAGED:
        return pg_compute()
    out = []
    for r in (SKR, SVR):
        out += [f"s_add_u32 s{r}, s{r}, %[kstep]", f"s_addc_u32 s{r + 1}, s{r + 1}, 0",
                f"s_sub_i32 s{r + 2}, s{r + 2}, %[kstep]", f"s_max_i32 s{r + 2}, s{r + 2}, 0"]
    return out


def vis_test(off):
    """vcc = key offset `off` (of this lane's keys in the tile) is visible to its row"""
    if LEFTWIN:   # (unsigned) off - LIML < wid <=> LIML <= off < LIML + wid = the right limit
        return [f"v_sub_u32 v{TW}, {off}, v{LIML}", f"v_cmp_lt_u32 vcc, v{TW}, %[wid]"]
    return [f"v_cmp_lt_i32 vcc, {off}, v{LIM}"]


def lim_step():
    return [f"v_add_u32 v{LIM}, -64, v{LIM}"] + ([f"v_add_u32 v{LIML}, -64, v{LIML}"] if LEFTWIN else [])


def softmax(dt, mask):
    """P = exp2(S c - m) of this lane's 32 scores (masked: keys at or past the lane's limit give
    0), the tile row sum in LT; 4 scores in flight"""
    ops = []
    for v in range(32):
        t = f"v{TMP + v % 8}"
        off, dword = value_info(v)
        ex = [f"v_exp_f32 {t}, {t}"]
        if mask:
            ex += vis_test(off) + [f"v_cndmask_b32 {t}, 0, {t}, vcc"]
        st = [[f"v_fma_f32 {t}, v{SBASE + v}, %[c], v{NM}"], ex,
              [f"v_mov_b32 v{LT}, {t}" if v == 0 else f"v_add_f32 v{LT}, v{LT}, {t}"]]
        if v & 1:
            st[2].append(f"v_cvt_pk_{dt}_f32 v{PBASE + dword}, v{TMP + (v - 1) % 8}, {t}")
        for k, txt in enumerate(st):
            ops.append((v + 2 * k, v, txt))
    out = []
    for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1])):
        out += txt
    return out + ["s_nop 0"]


def row_max(dst, raw=None):
    """masked max of this lane's row over the tile's 64 keys (both lane halves) -> dst (and the
    unmasked max -> raw)"""
    t2, ninf = f"v{MISC + 1}", f"v{MISC + 3}"
    out = [f"v_mov_b32 {ninf}, 0xff800000", f"v_mov_b32 {dst}, {ninf}"]
    if raw:
        out.append(f"v_mov_b32 {raw}, {ninf}")
    for v in range(32):
        off, _ = value_info(v)
        out += vis_test(off) + [f"v_cndmask_b32 {t2}, {ninf}, v{SBASE + v}, vcc",
                                f"v_max_f32 {dst}, {dst}, {t2}"]
        if raw:
            out.append(f"v_max_f32 {raw}, {raw}, v{SBASE + v}")
    out += [f"v_mov_b32 {t2}, {dst}", "s_nop 1", f"v_permlane32_swap_b32 {dst}, {t2}",
            "s_nop 1", f"v_max_f32 {dst}, {dst}, {t2}"]
    if raw:
        out += [f"v_mov_b32 {t2}, {raw}", "s_nop 1", f"v_permlane32_swap_b32 {raw}, {t2}",
                "s_nop 1", f"v_max_f32 {raw}, {raw}, {t2}"]
    return out


def first_max():
    """m = the masked max of tile 0 (in log2 units: NM = -c max; 0 for a row with no key).
    LEFTWIN: a row with no visible key in tile 0 (its window starts later) takes NM = +inf, so
    its first visible key gives P = inf and the redo path sets m to that tile's true max — the
    row's reference max is then exact, as tile 0's is for the others (a single-key row gets
    P = 1 and O = its V row bit for bit)"""
    mx, t2 = f"v{MISC}", f"v{MISC + 1}"
    if LEFTWIN:
        pinf = f"v{MISC + 3}"
        return XDL_NOPS + row_max(mx) + [
            f"v_mul_f32_e64 {t2}, -%[c], {mx}",
            f"v_cmp_lg_f32 vcc, 0xff800000, {mx}",
            f"v_mov_b32 {pinf}, 0x7f800000",           # (a literal and vcc: two constant-bus reads)
            f"v_cndmask_b32 v{NM}, {pinf}, {t2}, vcc"]
    return XDL_NOPS + row_max(mx) + [
        f"v_mul_f32_e64 {t2}, -%[c], {mx}",
        f"v_cmp_lg_f32 vcc, 0xff800000, {mx}",
        f"v_cndmask_b32 v{NM}, 0, {t2}, vcc"]


def redo_block(dt, uid):
    """rare path: the tile's scores passed the threshold against the reference m.  Take the
    tile's true (masked) max, m_new = max(m, c max); O and l scaled by 2^(m - m_new); the
    softmax redone against m_new (its row sum replaces LT).  Returns through SRA."""
    mx, t2, alpha = f"v{MISC}", f"v{MISC + 1}", f"v{MISC + 2}"
    out = [f".Lredo_{uid}:"] + XDL_NOPS
    if FEATURES:
        # in the true frame: this half's max lifted by its frame shift before the two lane
        # halves' maxima meet (causal linear ALiBi: the halves' keys differ by 4, SHIFT too;
        # SHIFT = 0 and NMTRUE = NM otherwise, bit for bit the plain path)
        ninf = f"v{MISC + 3}"
        out += [f"v_mov_b32 {ninf}, 0xff800000", f"v_mov_b32 {mx}, {ninf}"]
        for v in range(32):
            off, _ = value_info(v)
            out += vis_test(off) + [f"v_cndmask_b32 {t2}, {ninf}, v{SBASE + v}, vcc",
                                    f"v_max_f32 {mx}, {mx}, {t2}"]
        out += [f"v_fma_f32 {mx}, {mx}, %[c], v{SHIFT}",
                f"v_mov_b32 {t2}, {mx}", "s_nop 1", f"v_permlane32_swap_b32 {mx}, {t2}",
                "s_nop 1", f"v_max_f32 {t2}, {mx}, {t2}",
                f"v_max_f32_e64 {t2}, {t2}, -v{NMTRUE}",
                *([f"v_max_f32 {t2}, 0xff7fffff, {t2}"] if LEFTWIN else []),
                f"v_add_f32 {alpha}, v{NMTRUE}, {t2}",
                f"v_exp_f32_e64 {alpha}, -{alpha}",
                f"v_mul_f32 v{NMTRUE}, -1.0, {t2}",
                f"v_add_f32 v{NM}, v{NMTRUE}, v{SHIFT}",
                "s_nop 0",
                f"v_mul_f32 v{LRUN}, v{LRUN}, {alpha}"]
    else:
        out += row_max(mx)
        out += [f"v_mul_f32 {t2}, %[c], {mx}",
                f"v_max_f32_e64 {t2}, {t2}, -v{NM}",          # m_new = max(m_ref, c max)
                # (LEFTWIN: a row still at NM = +inf with no visible key here keeps m_new finite,
                # -FLT_MAX, so alpha = 2^(m - m_new) = 0, not NaN; its O and l are 0)
                *([f"v_max_f32 {t2}, 0xff7fffff, {t2}"] if LEFTWIN else []),
                f"v_add_f32 {alpha}, v{NM}, {t2}",             # m_new - m_ref >= 0
                f"v_exp_f32_e64 {alpha}, -{alpha}",
                f"v_mul_f32 v{NM}, -1.0, {t2}",
                "s_nop 0",
                f"v_mul_f32 v{LRUN}, v{LRUN}, {alpha}"]
    for i in range(64):
        t = f"v{TMP + i % 8}"
        out += [f"v_accvgpr_read_b32 {t}, a{ABASE_O + i}", f"v_mul_f32 {t}, {t}, {alpha}",
                f"v_accvgpr_write_b32 a{ABASE_O + i}, {t}"]
    out += ["s_nop 1"] + softmax(dt, True)
    return out + ["s_nop 3", f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]


def redo_check(uid, tag):
    """(inline part, stub): any lane's tile row sum past 2^slack -> the rare path; then l += LT"""
    inline = [f"v_cmp_lt_f32 vcc, %[thr], v{LT}", "s_nop 1", f"s_cbranch_vccnz .Lrc{tag}_{uid}",
              f".Lnr{tag}_{uid}:", f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}"]
    stub = [f".Lrc{tag}_{uid}:", f"s_getpc_b64 s[{SRA}:{SRA + 1}]", f".Lpc{tag}_{uid}:",
            f"s_add_u32 s{SRA}, s{SRA}, .Lnr{tag}_{uid} - .Lpc{tag}_{uid}",
            *addc_ret(SRA + 1, f".Lnr{tag}_{uid}", f".Lpc{tag}_{uid}", True),
            f"s_branch .Lredo_{uid}"]
    if "noredo" in ABL:
        return [f"v_add_f32 v{LRUN}, v{LRUN}, v{LT}"], []
    return inline, stub


def feat_call(uid, tag, block="feat"):
    """(inline part, stub): with any %[feat] bit set, a score-feature block (feature_block) over
    this tile's S before its max / softmax; returns through SRA"""
    if not FEATURES:
        return [], []
    inline = ["s_cmp_lg_u32 %[feat], 0", f"s_cbranch_scc1 .Lft{tag}_{uid}", f".Lfr{tag}_{uid}:"]
    stub = [f".Lft{tag}_{uid}:", f"s_getpc_b64 s[{SRA}:{SRA + 1}]", f".Lpf{tag}_{uid}:",
            f"s_add_u32 s{SRA}, s{SRA}, .Lfr{tag}_{uid} - .Lpf{tag}_{uid}",
            *addc_ret(SRA + 1, f".Lfr{tag}_{uid}", f".Lpf{tag}_{uid}", True),
            f"s_branch .L{block}_{uid}"]
    return inline, stub


def _softcap_ops():
    ops = []
    for v in range(32):
        sr = f"v{SBASE + v}"
        st_ = [[f"v_mul_f32 {sr}, %[scp2], {sr}"], [f"v_exp_f32 {sr}, {sr}"],
               [f"v_add_f32 {sr}, 1.0, {sr}"], [f"v_rcp_f32 {sr}, {sr}"],
               [f"v_fma_f32 {sr}, {sr}, -2.0, 1.0"]]
        for k, txt in enumerate(st_):
            ops.append((v + 2 * k, v, txt))
    return sum((txt for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1]))), [])


def _alibi_ops():
    import struct
    base = f"v{TMP + 7}"
    out = [f"s_add_i32 s{ST}, s{SJ}, 1", f"s_lshl_b32 s{ST}, s{ST}, 6", f"v_cvt_f32_i32 {base}, s{ST}",
           f"v_sub_f32 {base}, %[ald], {base}"]
    ops = []
    for v in range(32):
        off, _ = value_info(v)
        t = f"v{TMP + v % 7}"
        lit = "0x%08x" % struct.unpack("<I", struct.pack("<f", float(off)))[0]
        st_ = [[f"v_subrev_f32 {t}, {lit}, {base}"],
               [f"v_fma_f32 v{SBASE + v}, -%[alw], |{t}|, v{SBASE + v}"]]
        for k, txt in enumerate(st_):
            ops.append((v + 3 * k, v, txt))
    return out + sum((txt for _, _, txt in sorted(ops, key=lambda x: (x[0], x[1]))), [])


def _alibi_linear_ops():
    """causal ALiBi (every visible key <= pos + diag) as the reference kernel's linear bias
    +w key (mask_hip.h:163-164): S += w off per score (one v_fmac with the offset as a literal)
    and the tile's per-lane part w key0 folded into the exp argument: NM = NMTRUE + SHIFT with
    SHIFT = c w key0 = fma(%[alw2], 64 (j + 1), %[akb]) — the true -m stays in NMTRUE, so the
    shift never accumulates rounding"""
    import struct
    t = f"v{TMP + 7}"
    out = [f"s_add_i32 s{ST}, s{SJ}, 1", f"s_lshl_b32 s{ST}, s{ST}, 6", f"v_cvt_f32_i32 {t}, s{ST}",
           f"v_fma_f32 v{SHIFT}, %[alw2], {t}, %[ald]", f"v_add_f32 v{NM}, v{NMTRUE}, v{SHIFT}"]
    for v in range(32):
        off, _ = value_info(v)
        lit = "0x%08x" % struct.unpack("<I", struct.pack("<f", float(off)))[0]
        out.append(f"v_fmac_f32 v{SBASE + v}, {lit}, %[alw]")
    return out


def feature_block(uid):
    """the score features of the 8-wave kernel's transform (fmha_fwd_kernel.h transform_part),
    in place on this lane's 32 raw scores of tile j + 1 (SJ = j):
      bit 0 softcap: S = tanh(S pre) = 1 - 2 / (2^(2 log2e pre S) + 1)   (%[scp2] = 2 log2e pre)
      bit 1 ALiBi:   S -= w |pos + diag - key|   (%[alw] = slope / scale_softmax of the lane's
                     row, %[ald] = pos + diag - 4 hh; key = 64 (j + 1) + 4 hh + off)
    bit 2 causal ALiBi (wr = 0): _alibi_linear_ops, 1 VALU per score.
    5 VALU per score for the softcap, 2 for ALiBi, staggered over the scores.  Three entries,
    each returning via SRA: .Lfeat (both, by bit), .Lfsc (softcap by bit: tile 0 before its max)
    and .Lfal (ALiBi by bit: tile 0 after it)."""
    out = [f".Lfeat_{uid}:", "s_bitcmp1_b32 %[feat], 0", f"s_cbranch_scc0 .Lfa_{uid}"] + _softcap_ops()
    out += [f".Lfa_{uid}:", "s_bitcmp1_b32 %[feat], 2", f"s_cbranch_scc1 .Lfl_{uid}"]
    out += ["s_bitcmp1_b32 %[feat], 1", f"s_cbranch_scc0 .Lfe_{uid}"] + _alibi_ops()
    out += [f".Lfe_{uid}:", "s_nop 3", f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]
    out += [f".Lfl_{uid}:"] + _alibi_linear_ops() + ["s_nop 3", f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]
    out += [f".Lfsc_{uid}:", "s_bitcmp1_b32 %[feat], 0", f"s_cbranch_scc0 .Lfse_{uid}"] + _softcap_ops()
    out += [f".Lfse_{uid}:", "s_nop 3", f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]
    out += [f".Lfal_{uid}:", "s_bitcmp1_b32 %[feat], 2", f"s_cbranch_scc1 .Lfll_{uid}"]
    out += ["s_bitcmp1_b32 %[feat], 1", f"s_cbranch_scc0 .Lfle_{uid}"] + _alibi_ops()
    out += [f".Lfle_{uid}:", "s_nop 3", f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]
    out += [f".Lfll_{uid}:"] + _alibi_linear_ops() + ["s_nop 3", f"s_setpc_b64 s[{SRA}:{SRA + 1}]"]
    return out


def v_phase(dt, slot, kind, uid, tag, feat=True):
    """V phase: kind 'u' unmasked softmax, 'm' masked, 'n' none; DMA of the tile in slot.
    Returns (inline, out-of-line stubs)."""
    pieces = dma_pieces(slot)
    pre = pg_load() if PAGED else []
    if kind == "n" or ("nosm" in ABL and kind == "u"):
        return pre + sum(pieces, []) + dma_advance() + lim_step(), []
    sm = softmax(dt, kind == "m")
    fin, fstub = feat_call(uid, tag) if feat else ([], [])
    if DMAMIX:
        out = pre + pieces[0] + VPH_NOPS                # last QK^T results -> VALU
        # the other pieces spread through the softmax
        step = len(sm) // len(pieces)
        for n, pc in enumerate(pieces[1:]):
            at = (n + 1) * step + 3 * n
            sm[at:at] = pc
    else:
        out = pre + sum(pieces, []) + VPH_NOPS
    out += fin + sm
    inl, stub = redo_check(uid, tag)
    out += inl + dma_advance() + lim_step()
    return out, stub + fstub


ST_M, ST_MW, ST_V, ST_VW, ST_PRO, ST_TAIL, ST_EPI = range(7)


def st(k):
    """stamp: the cycles since the previous stamp go to class k (STAMPS builds only)"""
    if not STAMPS:
        return []
    return ["s_memtime s[96:97]", "s_waitcnt lgkmcnt(0)", "s_sub_u32 s99, s96, s98", "s_mov_b32 s98, s96",
            f"v_readlane_b32 s97, %[acc], {k}", "s_nop 3", "s_add_u32 s97, s97, s99", "s_nop 3",
            f"v_writelane_b32 %[acc], s97, {k}"]


def epilogue_core(dt):
    """O / l -> dt rows (16-byte stores after a permlane32 exchange), LSE; the row's two lane
    halves' sums combined first"""
    inv, L, t, lse, cls, pinf = (f"v{TMP + i}" for i in range(6))
    out = [f"v_mov_b32 {pinf}, 0x7f800000",
           f"v_mov_b32 {t}, v{LRUN}", "s_nop 1", f"v_permlane32_swap_b32 v{LRUN}, {t}", "s_nop 1",
           f"v_add_f32 {L}, v{LRUN}, {t}", f"v_rcp_f32 {inv}, {L}", f"v_log_f32 {lse}, {L}",
           f"v_mov_b32 {cls}, 0x63", f"v_cmp_class_f32 vcc, {L}, {cls}",
           f"v_cndmask_b32_e64 {inv}, {inv}, 1.0, vcc"]
    if EPI_SCALE:
        out.append(f"v_mul_f32 {inv}, {EPI_SCALE}, {inv}")
    out += [f"v_sub_f32 {lse}, {lse}, v{NM}",
           f"v_mul_f32 {lse}, 0x3f317218, {lse}", f"v_cndmask_b32 {lse}, {lse}, {pinf}, vcc",
           f"buffer_store_dword {lse}, %[loff], %[lsrd], 0 offen"]
    n = 0
    for d in range(4):
        for gp in (0, 2):
            vb = 0 if n % 2 == 0 else 16          # two alternating register sets in S
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


def epilogue(dt, tag=""):
    """once per wave: the rows' epilogue (marks SST).  Causal ALiBi in the linear frame (feat bit
    2): NM = NMTRUE + %[adiag] first, the -m of the kernels' |.| form, whose LSE the API converts
    to the reference's convention (fmha_lse_alibi_kernel) as for every other kernel"""
    fix = ([f"s_bitcmp1_b32 %[feat], 2", f"s_cbranch_scc0 .Lep{tag}_%=",
            f"v_add_f32 v{NM}, v{NMTRUE}, %[adiag]", f".Lep{tag}_%=:"] if FEATURES else [])
    return [f"s_mov_b32 s{SST}, 1"] + fix + XDL_NOPS + epilogue_core(dt)


N_EPI_STORES = 9       # 8 O row stores + the LSE store


def group_program(dt, grp):
    """the phase program of group A (grp 0) or B (grp 1); uid keeps their labels apart"""
    uid = f"{'AB'[grp]}_%="
    # tile t is published at the barrier closing global phase 2t-1: A (after V(t-2)) has loaded
    # through tile t-2+DLEAD, B (after M(t-2), its loads one phase later) through t-3+DLEAD
    m_wait = [f"s_waitcnt vmcnt({NPIECE * (DLEAD - 3)})"] if grp else []
    v_wait = [] if grp else [f"s_waitcnt vmcnt({NPIECE * (DLEAD - 2)})"]
    bar = ["s_barrier"]
    out, tail = [], []
    if FEATURES:
        out += [f"s_mov_b32 s{SJ}, -1"]                    # (tile j + 1 = 0 in the pre-loop phases)
    if grp:
        out += bar                                          # B runs one phase behind A
    # M(-1) = QK(0) (waves with a visible key), V(-1) = tile-0 max + softmax(0) (masked) + DMA
    out += st(ST_PRO) + [f"s_cmp_lt_i32 %[tw], 0", f"s_cbranch_scc1 .Lni_{uid}"]
    out += m_phase(dt, RING - 1, pv=False) + st(ST_M) + m_wait + bar + st(ST_MW)
    if FEATURES:
        # tile 0: the score features before its max (the V phase then runs none of its own)
        # ALiBi: tile 0's max is taken on the unbiased scores and lifted by the row's best bias
        # (%[alm] = -w * the distance from pos + diag to the row's nearest visible key), so the
        # reference max does not lag the diagonal (causal rows' scores rise along the keys)
        v, stub = v_phase(dt, DLEAD - 1, "m", uid, "f", feat=False)
        f0, s0 = feat_call(uid, "f0", "fsc")
        f1, s1 = feat_call(uid, "f1", "fal")
        out += XDL_NOPS + f0 + first_max() + [f"v_fma_f32 v{NM}, -%[c], %[alm], v{NM}",
                                               f"v_mov_b32 v{NMTRUE}, v{NM}"] + f1
        out += v + st(ST_V) + v_wait + bar
        stub += s0 + s1
    else:
        v, stub = v_phase(dt, DLEAD - 1, "m", uid, "f")
        out += first_max() + v + st(ST_V) + v_wait + bar
    tail += stub
    out += [f"s_branch .Lloop_{uid}", f".Lni_{uid}:"]
    # (no visible key: the same barriers and DMA duty)
    out += st(ST_M) + m_wait + bar + st(ST_MW)
    v, _ = v_phase(dt, DLEAD - 1, "n", uid, "fi")
    out += v + st(ST_V) + v_wait + bar
    out += [f".Lloop_{uid}:", f"s_mov_b32 s{SJ}, 0", f"s_cmp_ge_i32 s{SJ}, %[ntl]",
            f"s_cbranch_scc1 .Lexit_{uid}"]
    for ph in range(RING):
        vslot = (ph + DLEAD) % RING                          # the tile j+DLEAD this V phase loads
        out.append(f".Lph{ph}_{uid}:")
        out += st(ST_VW) + [f"s_cmp_ge_i32 s{SJ}, %[tw]", f"s_cbranch_scc1 .Lx{ph}_{uid}",
                f"s_add_i32 s{ST}, s{SJ}, 1"]
        if LEFTWIN:   # tile j+1 before the wave's first visible tile: an idle step (P(j) = 0)
            out += [f"s_cmp_lt_i32 s{ST}, %[fw]", f"s_cbranch_scc1 .Li{ph}_{uid}"]
        out += [f"s_cmp_lt_i32 s{ST}, %[ew]", f"s_cbranch_scc0 .Lm{ph}_{uid}"]
        if LEFTWIN:   # tiles before lw cross some row's left window edge
            out += [f"s_cmp_ge_i32 s{ST}, %[lw]", f"s_cbranch_scc0 .Lm{ph}_{uid}"]
        # unmasked step (inline)
        out += m_phase(dt, ph) + st(ST_M) + m_wait + bar + st(ST_MW)
        v, stub = v_phase(dt, vslot, "u", uid, f"u{ph}")
        out += v + st(ST_V) + v_wait + bar
        tail += stub
        out += [f".Lnx{ph}_{uid}:", f"s_add_i32 s{SJ}, s{SJ}, 1", f"s_cmp_ge_i32 s{SJ}, %[ntl]",
                f"s_cbranch_scc1 .Lexit_{uid}"]
        # masked step
        tail.append(f".Lm{ph}_{uid}:")
        tail += m_phase(dt, ph) + st(ST_M) + m_wait + bar + st(ST_MW)
        v, stub = v_phase(dt, vslot, "m", uid, f"m{ph}")
        tail += v + st(ST_V) + v_wait + bar + [f"s_branch .Lnx{ph}_{uid}"] + stub
        # j >= t_w: the last step (PV(j), then the epilogue beside the DMA) or an idle one
        tail += [f".Lx{ph}_{uid}:", f"s_cmp_eq_u32 s{SJ}, %[tw]", f"s_cbranch_scc0 .Li{ph}_{uid}"]
        tail += m_phase(dt, ph, qk=False) + st(ST_M) + m_wait + bar + st(ST_MW)
        v, _ = v_phase(dt, vslot, "n", uid, f"l{ph}")
        # DMA first, then the rows' stores (the youngest N_EPI_STORES may stay in flight)
        tail += v + st(ST_V) + epilogue(dt, f"{'AB'[grp]}{ph}") + st(ST_EPI)
        tail += ([] if grp else [f"s_waitcnt vmcnt({NPIECE * (DLEAD - 2) + N_EPI_STORES})"]) + bar
        tail += [f"s_branch .Lnx{ph}_{uid}"]
        tail.append(f".Li{ph}_{uid}:")
        tail += st(ST_M) + m_wait + bar + st(ST_MW)
        v, _ = v_phase(dt, vslot, "n", uid, f"i{ph}")
        tail += v + st(ST_V) + v_wait + bar + [f"s_branch .Lnx{ph}_{uid}"]
    out.append(f"s_branch .Lph0_{uid}")
    out.append(f".Lexit_{uid}:")
    out += st(ST_VW)
    if not grp:
        out += bar                                          # A's closing phase
    # rows that never reached a last step (no visible key): their O = 0, LSE = +inf
    out += [f"s_cmp_eq_u32 s{SST}, 0", f"s_cbranch_scc0 .Ldone_{uid}"] + epilogue(dt, f"{'AB'[grp]}x")
    out += [f".Ldone_{uid}:"] + ([] if "noepiwait" in ABL else ["s_waitcnt vmcnt(0)"])
    out += st(ST_TAIL) + ["s_branch .Lend_%="]
    return out + tail + redo_block(dt, uid) + (feature_block(uid) if FEATURES else [])


def item_program(dt):
    out = (["s_memtime s[96:97]", "s_waitcnt lgkmcnt(0)", "s_mov_b32 s98, s96"] if STAMPS else [])
    out += ["s_waitcnt lgkmcnt(0)",
           f"v_mov_b32 v{NM}, 0", f"v_mov_b32 v{LRUN}, 0", f"v_mov_b32 v{LIM}, %[lim]",
           *([f"v_mov_b32 v{LIML}, %[liml]"] if LEFTWIN else []),
           *([f"v_mov_b32 v{SHIFT}, 0", f"v_mov_b32 v{NMTRUE}, 0"] if FEATURES else []),
           f"s_mov_b32 s{SST}, 0"]
    if not ABL & {"nopro", "nopq"}:
        out += [f"buffer_load_dwordx4 {qtup(s)}, %[qoff], %[qsrd], 0 offen offset:{32 * s}" for s in range(8)]
    out += [f"v_accvgpr_write_b32 a{ABASE_O + i}, 0" for i in range(64)]
    if PAGED:     # tile 0's descriptors from its page; later tiles' at each V phase's end
        out += [f"s_mov_b32 s{SKR + 3}, 0x20000", f"s_mov_b32 s{SVR + 3}, 0x20000",
                f"s_mov_b32 s{SKEY}, %[skey0]"] + pg_load() + pg_compute()
    else:
        for r, lo, hi in ((SKR, "kblo", "kbhi"), (SVR, "vblo", "vbhi")):
            out += [f"s_mov_b32 s{r}, %[{lo}]", f"s_mov_b32 s{r + 1}, %[{hi}]",
                    f"s_mov_b32 s{r + 2}, %[kvbytes]", f"s_mov_b32 s{r + 3}, 0x20000"]
    for slot in range(DLEAD - 1):                            # tiles 0 .. DLEAD-2
        out += ([] if ABL & {"nopro", "nopkv"} else sum(dma_pieces(slot), []))
        out += (pg_load() if PAGED else []) + dma_advance()
    # Q and tile 0 landed, published
    w = NPIECE * (DLEAD - 2) if not ABL & {"nopro", "nopkv"} else 0
    if PRO_V0 and w:
        w += 2      # tile 0's two V pieces (issued after its K pieces) stay in flight: PV(0)
                    # comes after both groups' next vmcnt waits
    out += ([] if "nopro" in ABL else [f"s_waitcnt vmcnt({w})"]) + ["s_barrier"]
    out += ["s_cmp_eq_u32 %[grp], 0", "s_cbranch_scc0 .LgrpB_%="]
    out += group_program(dt, 0) + [".LgrpB_%=:"] + group_program(dt, 1) + [".Lend_%=:"]
    return out


SIG = ("const int kblo, const int kbhi, const int vblo, const int vbhi, const int kvbytes, "
       "const i32x4 qsrd, const i32x4 osrd, const i32x4 lsrd, const int kstep, const int kdst, "
       "const int ntl, const int tw, const int ew, const int grp, const float c, const float thr, "
       "const int kb0, const int kb1, const int vb0, const int vb1, const int dma0, const int dma1, "
       "const int lim, const int qoff, const int ooff, const int loff, const int feat, "
       "const float scp2, const float alw, const float ald, const float alm, const int lw, "
       "const int liml, const int wid, const int fw, const float alw2, const float adiag")
OPS = ['[kblo] "s"(kblo)', '[kbhi] "s"(kbhi)', '[vblo] "s"(vblo)', '[vbhi] "s"(vbhi)',
       '[kvbytes] "s"(kvbytes)', '[qsrd] "s"(qsrd)', '[osrd] "s"(osrd)', '[lsrd] "s"(lsrd)',
       '[kstep] "s"(kstep)', '[kdst] "s"(kdst)', '[ntl] "s"(ntl)', '[tw] "s"(tw)', '[ew] "s"(ew)',
       '[grp] "s"(grp)', '[c] "s"(c)', '[thr] "s"(thr)',
       '[kb0] "v"(kb0)', '[kb1] "v"(kb1)', '[vb0] "v"(vb0)', '[vb1] "v"(vb1)',
       '[dma0] "v"(dma0)', '[dma1] "v"(dma1)', '[lim] "v"(lim)', '[qoff] "v"(qoff)',
       '[ooff] "v"(ooff)', '[loff] "v"(loff)', '[feat] "s"(feat)', '[scp2] "s"(scp2)',
       '[alw] "v"(alw)', '[ald] "v"(ald)', '[alm] "v"(alm)', '[lw] "s"(lw)', '[liml] "v"(liml)',
       '[wid] "v"(wid)', '[fw] "s"(fw)', '[alw2] "v"(alw2)', '[adiag] "v"(adiag)']


def clobbers():
    regs = [f'"v{i}"' for i in range(100 if FEATURES else 98 if LEFTWIN else 96)] + [f'"a{i}"' for i in range(128)]
    regs += [f'"s{i}"' for i in range(SKR, SCM + 2)] + ([f'"s{i}"' for i in range(96, 100)] if STAMPS else [])
    return ", ".join(regs + ['"vcc"', '"scc"', '"memory"'])


SIG_PG = ", const int* btab, const int pstr, const int rowb, const int lgp, const int pmask, const int skv, const int skey0"
OPS_PG = ['[btab] "s"(btab)', '[pstr] "s"(pstr)', '[rowb] "s"(rowb)', '[lgp] "s"(lgp)', '[pmask] "s"(pmask)',
          '[skv] "s"(skv)', '[skey0] "s"(skey0)']


def emit(out=OUT):
    lines = [
        "// GENERATED by tools/gen_fwdpp.py -- do not edit by hand.",
        "// The 8-wave ping-pong D = 128 forward's item body (fmha_fwdpp_kernel.h): one asm statement",
        "// per dtype with a fixed register map; see the generator's docstring for the schedule.",
        "#pragma once",
        '#include "fmha_common.h"',
        "",
        *(["#define XFA_FWDPP_STAMPS 1           // diagnostic build (--stamps)"] if STAMPS else []),
        "namespace xfa {",
        "typedef __attribute__((ext_vector_type(4))) int i32x4;",
        f"constexpr int kFwdppRing = {RING};           // K / V tile slots the body addresses",
        "",
    ]
    global PAGED
    # the dense body, then (not in stamps builds) the paged-K/V body
    for paged, dt in [(False, "bf16"), (False, "f16")] + ([] if STAMPS else [(True, "bf16"), (True, "f16")]):
        PAGED = paged
        prog = item_program(dt)
        PAGED = False
        prog += GUARDS
        GUARDS.clear()
        sig = SIG + (SIG_PG if paged else "") + (", unsigned& acc" if STAMPS else "")
        lines.append(f"__device__ __forceinline__ void fwdpp{'_pg' if paged else ''}_item_{dt}({sig}) {{")
        lines.append("    asm volatile(")
        lines += [f'        "{b}\\n"' for b in prog]
        lines.append('        : [acc] "+v"(acc)' if STAMPS else "        :")
        lines.append("        : " + ",\n          ".join(OPS + (OPS_PG if paged else [])))
        lines.append(f"        : {clobbers()});")
        lines.append("}")
        lines.append("")
        print(dt, "paged" if paged else "", len(prog), "instructions/labels")
    lines.append("}  // namespace xfa")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--abl", default="", help="timing ablations, comma list (results invalid)")
    ap.add_argument("--stamps", action="store_true", help="diagnostic phase stamps (XFA_FWDPP_STAMPS)")
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--pro-v0", action="store_true", help="prologue waits for Q and K0 only")
    a = ap.parse_args()
    PRO_V0 = a.pro_v0
    ABL = set(x for x in a.abl.split(",") if x)
    STAMPS = a.stamps
    emit(a.out)

"""LDS bank cycles of the backward's dS^T traffic (D = 128: 8 waves x 32 keys): the bf16 dS^T
stores (ds_write_b64, 4 groups of 16 contiguous lanes, 32 banks) and the dQ phase's
transposed reads (ds_read_b64_tr_b16, 2 x 32 lanes, 64 banks), under round 3's image and the
current fmha_bwd_kernel.h ds_off (lane groups: MI355X_MICROARCH.md § LDS).

  python tools/bwd_banks.py
"""


def round3(row, col):
    return row * 64 + (((col >> 3) ^ (((row >> 3) & 1) << 1)) << 4) + ((col >> 2) & 1) * 8


def current(row, col):
    s1 = (((row >> 3) & 1) << 1) | ((row >> 1) & 1)
    s0 = (row >> 2) & 1
    return row * 64 + (((col >> 3) ^ s1) << 4) + ((((col >> 2) & 1) ^ s0) << 3)


def cycles(addrs, groups, width, nbanks):
    tot = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for w in range(width // 4):
                banks.setdefault((a // 4 + w) % nbanks, set()).add(a // width)
        tot += max(len(v) for v in banks.values())
    return tot


if __name__ == "__main__":
    for name, f in (("round 3", round3), ("current", current)):
        st = [cycles([f(w * 32 + (l & 31), 8 * gq + 4 * (l >> 5)) for l in range(64)],
                     [list(range(16 * j, 16 * j + 16)) for j in range(4)], 8, 32)
              for w in range(8) for gq in range(4)]
        rd = [cycles([ks * 32 * 64 + f(8 * (l >> 4) + ((l & 15) >> 2) + 4 * part, 16 * mt + 4 * (l & 3))
                      for l in range(64)], [list(range(32)), list(range(32, 64))], 8, 64)
              for mt in range(2) for part in range(2) for ks in range(8)]
        for r in range(64):
            assert sorted((f(r, c) - r * 64) // 8 for c in range(0, 32, 4)) == list(range(8))
        print(f"{name:8s} dS^T ds_write_b64 {sum(st) / len(st):.1f} cycles (4 ideal)   "
              f"dQ ds_read_b64_tr_b16 {sum(rd) / len(rd):.1f} (2 ideal)")

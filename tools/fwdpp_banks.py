"""LDS bank cycles of the ping-pong forward's fragment reads (csrc/fmha_fwdpp_kernel.h) under the
kv_off image with the chunk XORed by row bits 2-3 through a map F (the 32x32 body: identity; the
16x16 body: ppx16 = 0, 2, 3, 1), from the lane groups and bank functions of
MI355X_MICROARCH.md § LDS (tools/decode_banks.py): ds_read_b128 4 groups of 16 lanes, 64 banks;
ds_read_b64_tr_b16 2 x 32 lanes, 64 banks.

  python tools/fwdpp_banks.py          (every F: the 16x16 reads are conflict-free for 4 of 24)
"""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from decode_banks import B128, HALVES, cycles  # noqa: E402

HD = 128


def image(F):
    return lambda r, c: 16 * HD * (r >> 3) + 512 * (c >> 2) + 64 * (r & 7) + 16 * ((c & 3) ^ F[(r >> 2) & 3])


def body32(F):
    off = image(F)
    k = [cycles([off((l & 31) + 32 * kt, 2 * u + (l >> 5) + 4 * s) for l in range(64)], B128, 16, 64)
         for kt in range(2) for u in range(2) for s in range(4)]

    def va(l, u, dt):
        hh, q4 = l >> 5, (l & 15) >> 2
        col = 16 * ((l >> 4) & 1) + 4 * (l & 3) + 32 * dt
        return off(8 * u + 4 * hh + q4, col >> 3) + 8 * ((col >> 2) & 1)
    v = [cycles([va(l, u, dt) for l in range(64)], HALVES, 8, 64) for u in range(2) for dt in range(4)]
    return sum(k) / len(k), sum(v) / len(v)


def body16(F):
    off = image(F)
    k = [cycles([off(16 * kt + (l & 15), 4 * s + (l >> 4)) for l in range(64)], B128, 16, 64)
         for kt in range(4) for s in range(4)]

    def va(l, e, ks, h, dth):
        g, q4, p4 = l >> 4, (l & 15) >> 2, l & 3
        return off(4 * g + q4 + 32 * ks + 16 * h, 4 * dth + 2 * e + (p4 >> 1)) + 8 * (p4 & 1)
    v = [cycles([va(l, e, ks, h, dth) for l in range(64)], HALVES, 8, 64)
         for e in range(2) for ks in range(2) for h in range(2) for dth in range(4)]
    return sum(k) / len(k), sum(v) / len(v)


if __name__ == "__main__":
    print("cycles per instruction (ideal: K ds_read_b128 4, V^T ds_read_b64_tr_b16 2)")
    print("32x32 body, F = identity:", body32([0, 1, 2, 3]))
    for F in itertools.permutations(range(4)):
        print("16x16 body, F =", F, body16(list(F)), "<- ppx16" if F == (0, 2, 3, 1) else "")

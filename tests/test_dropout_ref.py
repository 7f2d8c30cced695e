"""CPU: the dropout RNG restatement (oracle/dropout_ref.py) against a scalar transcription of
the reference's Philox (csrc/flash_attn/src/philox.cuh:32-50: mulhilo32, six rounds with Weyl
key bumps plus the final round), and the layout of the keep mask."""
import random

import numpy as np

from oracle import dropout_ref as drf


def _philox_scalar(seed, subsequence, offset):
    """philox.cuh's philox(seed, subsequence, offset) on Python ints (the counter's low 64 bits
    are `offset`, the high 64 `subsequence`; key = seed's two 32-bit halves)."""
    m32 = 0xFFFFFFFF
    key = [seed & m32, seed >> 32]
    ctr = [offset & m32, offset >> 32, subsequence & m32, subsequence >> 32]

    def rnd(c, k):
        r0 = 0xD2511F53 * c[0]
        r1 = 0xCD9E8D57 * c[2]
        return [((r1 >> 32) ^ c[1] ^ k[0]) & m32, r1 & m32, ((r0 >> 32) ^ c[3] ^ k[1]) & m32, r0 & m32]
    for _ in range(6):
        ctr = rnd(ctr, key)
        key = [(key[0] + 0x9E3779B9) & m32, (key[1] + 0xBB67AE85) & m32]
    return rnd(ctr, key)


def test_vectorised_philox_is_the_reference_algorithm():
    rng = random.Random(0)
    for _ in range(200):
        seed, sub, off = rng.getrandbits(64), rng.getrandbits(64), rng.getrandbits(64)
        want = _philox_scalar(seed, sub, off)
        c = [off & 0xFFFFFFFF, off >> 32, sub & 0xFFFFFFFF, sub >> 32]
        got = drf.philox4x32_7(seed & 0xFFFFFFFF, seed >> 32, *[np.uint32(x) for x in c])
        assert [int(x) for x in got] == want


def test_keep_mask_layout_and_rate():
    seed, offset, p = 1234567, 89, 0.3
    m = drf.keep_mask(seed, offset, 2, 3, 37, 45, p)
    assert m.shape == (2, 3, 37, 45)
    # element (b, h, pos, key) = byte key & 3 of word pos & 3 of block (pos >> 2, key >> 2)
    b, h, pos, key = 1, 2, 22, 41
    w = drf.philox4x32_7(seed & 0xFFFFFFFF, (seed >> 32) ^ (offset >> 32), np.uint32(key >> 2),
                         np.uint32(pos >> 2), np.uint32(b * 3 + h), np.uint32(offset))
    byte = (int(w[pos & 3]) >> (8 * (key & 3))) & 0xFF
    assert m[b, h, pos, key] == (byte <= drf.keep_threshold(p))
    big = drf.keep_mask(7, 0, 1, 4, 256, 256, p)
    assert abs((1 - big.mean()) - p) < 0.01

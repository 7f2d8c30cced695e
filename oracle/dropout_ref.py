"""CPU restatement of the dropout keep bits — TEST INFRASTRUCTURE ONLY (the product never
imports oracle/).

The reference draws dropout with Philox4x32 (seven rounds: `philox()` in
csrc/flash_attn/src/philox.cuh:32-50, six rounds plus the final one, Weyl key bumps) and keeps
a score iff its random byte <= floor((1 - p_dropout) * 255) (dropout_hip.h:58-63 with
paged_attn.cpp:106-113).  Its counter layout follows its MMA tiling, which gfx950 does not
share (bit-compatibility with the DCU RNG layout is not a goal), so this build
fixes its own layout (xf_flash_attention_cutlass_amd/csrc/fmha_common.h drop_block):

  block (pos >> 2, key >> 2) of (batch x head) bh = b * H + h:
    words = philox4x32_7(key = (seed_lo, seed_hi ^ offset_hi),
                         counter = (key >> 2, pos >> 2, bh, offset_lo))
  keep(pos, key) = byte (key & 3) of word (pos & 3)  <=  keep_thr

This module computes the same bits with numpy, so a test can check the kernels' masks bit for
bit (tests/test_dropout_gpu.py) — parity of the RNG is pinned by this restatement of the
published Philox algorithm, not by reference outputs (the reference's dropout path never runs
on its C ABI).
"""
from __future__ import annotations

import math

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_LO = np.uint64(0xFFFFFFFF)


def philox4x32_7(k0, k1, c0, c1, c2, c3):
    """Vectorised Philox4x32-7 (uint32 arrays, broadcast); returns the 4 output words."""
    k0, k1 = np.uint32(k0), np.uint32(k1)
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32) for x in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    with np.errstate(over="ignore"):
        for _ in range(7):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            n0 = (p1 >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0
            n2 = (p0 >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1
            c0, c1, c2, c3 = n0, (p1 & _LO).astype(np.uint32), n2, (p0 & _LO).astype(np.uint32)
            k0 = np.uint32(int(k0) + int(_W0) & 0xFFFFFFFF)
            k1 = np.uint32(int(k1) + int(_W1) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def keep_threshold(p_dropout: float) -> int:
    return int(math.floor((1.0 - p_dropout) * 255.0))


def keep_mask(seed: int, offset: int, b: int, h: int, sq: int, sk: int, p_dropout: float):
    """bool [b, h, sq, sk]: True = kept."""
    seed, offset = int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1)
    k0 = seed & 0xFFFFFFFF
    k1 = ((seed >> 32) ^ (offset >> 32)) & 0xFFFFFFFF
    nqb, nkb = (sq + 3) // 4, (sk + 3) // 4
    bh = np.arange(b * h, dtype=np.uint32).reshape(-1, 1, 1)
    qb = np.arange(nqb, dtype=np.uint32).reshape(1, -1, 1)
    kb = np.arange(nkb, dtype=np.uint32).reshape(1, 1, -1)
    words = philox4x32_7(k0, k1, kb, qb, bh, np.uint32(offset & 0xFFFFFFFF))
    w = np.stack(words, axis=2)                       # [bh, qb, 4 (pos & 3), kb]
    bytes_ = np.stack([(w >> np.uint32(8 * j)) & np.uint32(0xFF) for j in range(4)], axis=-1)
    # [bh, qb, pos & 3, kb, key & 3] -> [bh, q, k]
    m = bytes_.reshape(b * h, nqb * 4, nkb * 4)[:, :sq, :sk] <= keep_threshold(p_dropout)
    return m.reshape(b, h, sq, sk)

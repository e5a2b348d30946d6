"""Independent numpy restatement of the RAID5/RAID6 arithmetic (ORACLE, test-only).

Second, independent path next to the C restatement in ``isal_oracle.c``:
it builds GF(2^8) products by carry-less "Russian peasant" multiplication
(no log/antilog tables, no Horner form) so a shared mistake between the two
restatements is unlikely.  Semantics follow isa-l v2.30.0 as the reference
uses it:

* ``xor_gen``  -- P = XOR_j D_j                     (raid5_simple.c:154,176)
* ``pq_gen``   -- P = XOR_j D_j, Q = XOR_j 2^j D_j  (gf_vect_mul.c:152-169)
* recovery      -- gf_vect_mul.c:242-347, raid5.c:544-594

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg may use
this module.
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D


def _peasant(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= POLY
        b >>= 1
    return r


MUL = np.array([[_peasant(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
INV = np.zeros(256, dtype=np.uint8)
for _a in range(1, 256):
    INV[_a] = int(np.nonzero(MUL[_a] == 1)[0][0])


def gf_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gf_inv(a: int) -> int:
    return int(INV[a])


def gf_pow2(e: int) -> int:
    e %= 255
    r = 1
    for _ in range(e):
        r = _peasant(r, 2)
    return r


def gf_vect_mul_init(c: int) -> np.ndarray:
    """The 32-byte nibble table isa-l's gf_vect_mul_init produces."""
    lo = MUL[c, np.arange(16)]
    hi = MUL[c, np.arange(16) << 4]
    return np.concatenate([lo, hi]).astype(np.uint8)


def mul_vec(c: int, x: np.ndarray) -> np.ndarray:
    return MUL[c][x]


def xor_gen(data: np.ndarray) -> np.ndarray:
    """data: [k, len] uint8 -> P [len]."""
    return np.bitwise_xor.reduce(data, axis=0)


def pq_gen(data: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """data: [k, len] uint8 -> (P, Q), Q = XOR_j 2^j D_j by direct products."""
    p = np.bitwise_xor.reduce(data, axis=0)
    q = np.zeros(data.shape[1], dtype=np.uint8)
    for j in range(data.shape[0]):
        q ^= MUL[gf_pow2(j)][data[j]]
    return p, q


def recover(strips: np.ndarray, k: int, m: int, fail: list[int]) -> np.ndarray:
    """strips: [k+m, len] (lost rows hold garbage) -> copy with lost rows rebuilt."""
    out = strips.copy()
    data_lost = sorted(f for f in fail if f < k)
    alive = [j for j in range(k) if j not in data_lost]
    ps = np.zeros(strips.shape[1], dtype=np.uint8)
    qs = np.zeros(strips.shape[1], dtype=np.uint8)
    for j in alive:
        ps ^= strips[j]
        qs ^= MUL[gf_pow2(j)][strips[j]]
    lost_p = k in fail
    lost_q = m == 2 and (k + 1) in fail
    if len(data_lost) == 0:
        if lost_p:
            out[k] = ps
        if lost_q:
            out[k + 1] = qs
    elif len(data_lost) == 1:
        x = data_lost[0]
        if not lost_p:
            out[x] = strips[k] ^ ps
            if lost_q:
                out[k + 1] = qs ^ MUL[gf_pow2(x)][out[x]]
        else:
            out[x] = MUL[gf_pow2(255 - x)][strips[k + 1] ^ qs]
            out[k] = ps ^ out[x]
    else:
        x, y = data_lost
        pxy = strips[k] ^ ps
        qxy = strips[k + 1] ^ qs
        gyx = gf_pow2(y - x)
        den = gf_inv(gyx ^ 1)
        a = gf_mul(gyx, den)
        b = gf_mul(gf_pow2(255 - x), den)
        out[x] = MUL[a][pxy] ^ MUL[b][qxy]
        out[y] = pxy ^ out[x]
    return out

"""GPU tests of the host-resident stripe path (draid_ec_host_*): stripes in
pinned host memory, copied in / encoded or rebuilt in HBM / copied out,
bit-exact against the oracle."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _host_batch(k, m, L, B, gap, seed):
    n = k + m
    ss = n * (L + gap) + 64
    t = torch.zeros(B * ss, dtype=torch.uint8).pin_memory()
    a = t.numpy()
    rng = np.random.default_rng(seed)
    for s in range(B):
        for j in range(k):
            o = s * ss + j * (L + gap)
            a[o:o + L] = rng.integers(0, 256, L, dtype=np.uint8)
    return t, a, L + gap, ss


def _strips(a, k, m, L, B, st, ss):
    return np.stack([np.stack([a[s * ss + j * st: s * ss + j * st + L] for j in range(k + m)])
                     for s in range(B)])


@pytest.mark.parametrize("k,m,L,B,gap,chunk", [(8, 2, 65536, 40, 0, 0), (4, 1, 4096, 9, 512, 2),
                                               (16, 2, 8192, 5, 0, 1), (8, 2, 1000, 13, 24, 4)])
def test_host_encode_reconstruct(ec, k, m, L, B, gap, chunk):
    t, a, st, ss = _host_batch(k, m, L, B, gap, seed=L + B)
    before = _strips(a, k, m, L, B, st, ss).copy()
    assert ec.host_encode(t, k, m, L, B, st, ss, chunk) == 0
    got = _strips(a, k, m, L, B, st, ss)
    ref = before.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, (k + m) * L) == 0
    assert (got == ref).all()
    # gaps untouched
    if gap:
        assert not a[st - gap + 0: st].any()
    rng = np.random.default_rng(B)
    fail = np.full((B, 2), 0xFF, np.uint8)
    for s in range(B - 1):  # the last stripe has nothing to rebuild
        nf = int(rng.integers(1, m + 1))
        fail[s, :nf] = rng.choice(k + m, nf, replace=False)
        for j in map(int, fail[s, :nf]):
            a[s * ss + j * st: s * ss + j * st + L] = 0xEE
    ftab = fail.reshape(-1).copy()
    assert ec.host_reconstruct(t, k, m, L, B, st, ss, ftab.ctypes.data, chunk) == 0
    assert (_strips(a, k, m, L, B, st, ss) == ref).all()

"""Strips in pinned HOST memory through a context that resolves host pointers (what the
raid module's channels do with SPDK buffers).  Such launches run the work lists' looping
kernels -- one wave per item, one workgroup per CU, every workgroup striding over the work
items -- at every stripe width, so each case here queues more work items than the GPU has
CUs: the loops loop.  Bit-exact against the oracle, as everywhere."""
import numpy as np
import pytest
import torch

import oracle
from test_gpu_sg import Pool, _fill

pytestmark = pytest.mark.gpu

WIDTHS = [(2, 1), (3, 1), (4, 1), (8, 1), (13, 1), (20, 1), (24, 1),
          (2, 2), (3, 2), (4, 2), (5, 2), (7, 2), (8, 2), (9, 2), (10, 2), (12, 2), (16, 2),
          (20, 2), (21, 2), (32, 2), (40, 2)]


def _pinned(nbytes):
    t = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    return t, t.numpy()


@pytest.mark.parametrize("k,m", WIDTHS)
def test_whole_strips_in_host_memory(ec, k, m):
    """Aligned strips of 12 KiB + 48 bytes (vector path with a short last chunk), 40
    stripes = 520 work items; every stripe loses one or two random strips."""
    L, B = 12 * 1024 + 48, 40
    n = k + m
    rng = np.random.default_rng(900 + 10 * k + m)
    t, a = _pinned(B * n * L)
    a[:] = 0
    view = a.reshape(B, n, L)
    view[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    ref = a.copy()
    assert oracle.encode_strided(ref, k, m, L, B, L, n * L) == 0
    base = t.data_ptr()
    strips = [[[(base + (s * n + j) * L, L)] for j in range(n)] for s in range(B)]
    ctx = ec.Ctx()
    try:
        ctx.set_host_pointers(True)
        for s in range(B):
            assert ctx.encode_sg(k, m, strips[s], L) == 0
        ctx.flush()
        ctx.synchronize()
        assert (a == ref).all()
        fails = []
        for s in range(B):
            f = sorted(rng.choice(n, int(rng.integers(1, m + 1)), replace=False).tolist())
            fails.append(f)
            for j in f:
                view[s, j] = 0xA5
        for s in range(B):
            assert ctx.reconstruct_sg(k, m, strips[s], L, fails[s]) == 0
        ctx.flush()
        ctx.synchronize()
        bad = [(s, fails[s]) for s in range(B) if not (view[s] == ref.reshape(B, n, L)[s]).all()]
        assert not bad, bad[:4]
    finally:
        ctx.close()


@pytest.mark.parametrize("k,m,L,B", [(4, 1, 4096, 70), (8, 2, 8192 + 48, 40), (16, 2, 3000, 90),
                                     (11, 2, 777, 300), (3, 2, 5000, 60)])
def test_scattered_pieces_in_host_memory(ec, k, m, L, B):
    """Misaligned pieces, zero-length iovecs and prefixes (byte path, uneven segment
    lengths: an explicit work list), more work items than CUs."""
    rng = np.random.default_rng(k * L + B)
    pool = Pool(rng, k, m, L, B, prefix=True)
    _fill(pool, rng)
    t, a = _pinned(pool.size)
    a[:] = pool.host
    base = t.data_ptr()
    ctx = ec.Ctx()
    try:
        ctx.set_host_pointers(True)
        for s in range(B):
            assert ctx.encode_sg(k, m, pool.strips(base, s), L, pool.offsets[s]) == 0
        ctx.flush()
        ctx.synchronize()
        got = a.copy()
        ref = np.stack([np.stack([pool.gather(pool.host, s, j) for j in range(k + m)])
                        for s in range(B)])
        assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, (k + m) * L) == 0
        for s in range(B):
            for j in range(k + m):
                assert (pool.gather(got, s, j) == ref[s, j]).all(), (s, j)
        fails = []
        for s in range(B):
            f = sorted(rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False).tolist())
            fails.append(f)
            for j in f:
                pool.scatter(a, s, j, np.full(L, 0x5A, np.uint8))
        for s in range(B):
            assert ctx.reconstruct_sg(k, m, pool.strips(base, s), L, fails[s],
                                      pool.offsets[s]) == 0
        ctx.flush()
        ctx.synchronize()
        for s in range(B):
            for j in range(k + m):
                assert (pool.gather(a, s, j) == ref[s, j]).all(), (s, j, fails[s])
    finally:
        ctx.close()


@pytest.mark.parametrize("nd", [1, 2, 3])
@pytest.mark.parametrize("k,m", [(4, 1), (8, 2), (16, 2), (40, 2)])
def test_rmw_update_in_host_memory(ec, k, m, nd):
    """The read-modify-write update's looping form: 80 stripes x 5 chunks = 400 work
    items, whole strips of 4 KiB + 21 bytes (vectors and a ragged tail), odd stripes at a
    3-byte offset (byte path)."""
    L, B = 4096 + 21, 80
    n = k + m
    rng = np.random.default_rng(5000 + 10 * k + nd)
    pad = 16
    t, a = _pinned(B * n * (L + pad))
    tn, an = _pinned(B * k * (L + pad))
    to, ao = _pinned(B * k * (L + pad))
    a[:] = 0
    stripes = a.reshape(B, n, L + pad)
    new = an.reshape(B, k, L + pad)
    old = ao.reshape(B, k, L + pad)
    off = [0 if s % 2 == 0 else 3 for s in range(B)]
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    enc = np.zeros((B, n, L), np.uint8)
    enc[:, :k] = data
    assert oracle.encode_strided(enc.reshape(-1), k, m, L, B, L, n * L) == 0
    newdata = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    for s in range(B):
        o = off[s]
        stripes[s, :, o:o + L] = enc[s]
        old[s, :, o:o + L] = data[s]
        new[s, :, o:o + L] = newdata[s]
    expect = enc.copy()
    ctx = ec.Ctx()
    try:
        ctx.set_host_pointers(True)
        for s in range(B):
            o = off[s]
            idx = [(s + 5 * x) % k for x in range(nd)]
            if len(set(idx)) != nd:
                idx = [(s + x) % k for x in range(nd)]
            adr = lambda tt, row, i: tt.data_ptr() + ((s * row + i) * (L + pad)) + o  # noqa: E731
            olds = [[(adr(to, k, i), L)] for i in idx]
            news = [[(adr(tn, k, i), L)] for i in idx]
            par = [[(adr(t, n, k + j), L)] for j in range(m)]
            assert ctx.update_sg(k, m, idx, olds, news, par, L) == 0
            for i in idx:
                expect[s, i] = newdata[s, i]
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()
    ref = expect.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    for s in range(B):
        o = off[s]
        assert (stripes[s, k:, o:o + L] == ref[s, k:]).all(), s
        assert (stripes[s, :k, o:o + L] == enc[s, :k]).all(), s   # the update touches parity only

"""Concurrency: SPDK calls the parity path from several reactor threads at once.
The isa-l-shaped synchronous calls (per-thread stream) and per-thread contexts
must give the oracle's bytes when driven from many host threads together."""
import threading

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_sync_calls_from_many_threads(ec):
    k, L, T, reps = 8, 65536, 8, 20
    n = k + 2
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    bufs = [torch.randint(0, 256, (n, L), dtype=torch.uint8, device=DEV, generator=g)
            for _ in range(T)]
    for b in bufs:
        b[k:] = 0
    errors = []

    def worker(t):
        try:
            b = bufs[t]
            ptrs = [b[j].data_ptr() for j in range(n)]
            for _ in range(reps):
                assert ec.pq_gen(ptrs, L) == 0
                assert ec.pq_check(ptrs, L) == 0
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for b in bufs:
        got = b.cpu().numpy()
        ref = got.copy()
        assert oracle.encode_strided(ref.reshape(-1), k, 2, L, 1, L, n * L) == 0
        assert (got == ref).all()


def test_contexts_on_many_threads(ec):
    """One context per thread (one per io_channel), each queueing its own stripes
    and flushing concurrently."""
    k, m, L, B, T = 8, 2, 16384, 64, 6
    n = k + m
    g = torch.Generator(device=DEV)
    g.manual_seed(4)
    bufs = [torch.randint(0, 256, (B, n, L), dtype=torch.uint8, device=DEV, generator=g)
            for _ in range(T)]
    for b in bufs:
        b[:, k:] = 0
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    errors = []

    def worker(t):
        try:
            b = bufs[t]
            base = b.data_ptr()
            ctx = ec.Ctx()
            try:
                for rep in range(3):
                    for s in range(B):
                        strips = [[(base + (s * n + j) * L, L)] for j in range(n)]
                        assert ctx.encode_sg(k, m, strips, L) == 0
                    ctx.flush()
                ctx.synchronize()
            finally:
                ctx.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for b in bufs:
        got = b.cpu().numpy()
        ref = got.copy()
        assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
        assert (got == ref).all()


def test_pageable_memory_from_many_threads(ec):
    """The relinked reference calls the isa-l names on malloc'd memory from every reactor:
    each thread bounces its vectors through its own pinned arena and its host stripes
    through its own pair of pinned buffers.  Eight threads at once, sizes on both sides of
    the arena limit, every byte against the oracle."""
    k, T, reps = 8, 8, 6
    n = k + 2
    rng = np.random.default_rng(11)
    lens = [4096, 65536, 4096, 1 << 20, 65536, 4096, 65536, 1 << 20]  # 1 MiB x 10: device arena
    vecs = [[rng.integers(0, 256, lens[t], dtype=np.uint8) for _ in range(n)] for t in range(T)]
    S, B = 32768, 40
    stripes = [rng.integers(0, 256, B * n * S, dtype=np.uint8) for _ in range(T)]
    fails = [np.stack([np.arange(B) % n, (np.arange(B) + 1 + t) % n], axis=1).astype(np.uint8)
             for t in range(T)]
    for f in fails:
        f[f[:, 0] == f[:, 1], 1] = 0xFF
    want = []
    for t in range(T):
        ref = np.concatenate(vecs[t]).copy()
        assert oracle.encode_strided(ref, k, 2, lens[t], 1, lens[t], n * lens[t]) == 0
        sref = stripes[t].copy()
        assert oracle.encode_strided(sref, k, 2, S, B, S, n * S) == 0
        want.append((ref, sref))
    errors = []

    def worker(t):
        try:
            L = lens[t]
            ptrs = [v.ctypes.data for v in vecs[t]]
            for _ in range(reps):
                vecs[t][k][:] = 0
                vecs[t][k + 1][:] = 0
                assert ec.pq_gen(ptrs, L) == 0
                assert ec.pq_check(ptrs, L) == 0
                lost = vecs[t][1].copy()
                vecs[t][1][:] = 0x33
                assert ec.recover(k, 2, L, ptrs, [1]) == 0
                assert (vecs[t][1] == lost).all()
            a = stripes[t]
            assert ec.host_encode(a.ctypes.data, k, 2, S, B, S, n * S) == 0
            enc = a.copy()
            view = a.reshape(B, n, S)
            for s in range(B):
                for f in fails[t][s]:
                    if f != 0xFF:
                        view[s, f] = 0x77
            assert ec.host_reconstruct(a.ctypes.data, k, 2, S, B, S, n * S,
                                       fails[t].ctypes.data) == 0
            assert (a == enc).all()
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in range(T):
        assert (np.concatenate(vecs[t]) == want[t][0]).all(), t
        assert (stripes[t] == want[t][1]).all(), t

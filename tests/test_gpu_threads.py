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

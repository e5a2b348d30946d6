"""Contracts of the scatter-gather context that an SPDK module relies on:

* groups of one flush run in the order their first segment was queued, also when
  a group object of an earlier batch exists (a reconstruct into chunk buffers,
  then an encode that reads them: raid5.c's degraded write shape);
* a flush that fails part-way keeps exactly the unlaunched segments queued;
* tickets complete per flush; host pointers of pinned memory are resolved by the
  context.
Bit-exact against the CPU oracle.
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def stripes(k, m, L, B, seed):
    rng = np.random.default_rng(seed)
    a = np.zeros((B, k + m, L), np.uint8)
    a[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    ref = a.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, (k + m) * L) == 0
    return a, ref


def runs(t, s, n):
    """One iovec per strip of stripe s of the [B, n, L] device tensor t."""
    L = t.shape[2]
    return [[(t[s, j].data_ptr(), L)] for j in range(n)]


def test_groups_run_in_queue_order_of_the_current_batch(ec):
    k, m, L, B = 4, 2, 4096, 8
    n = k + m
    a, ref = stripes(k, m, L, B, 1)
    ctx = ec.Ctx()
    try:
        # batch 1 creates the ENCODE group first (so it is the older group object)
        d = torch.from_numpy(a).to(DEV)
        torch.cuda.synchronize()
        for s in range(B):
            ctx.encode_sg(k, m, runs(d, s, n), L)
        ctx.flush()
        ctx.synchronize()
        assert (d.cpu().numpy() == ref).all()
        # batch 2: lose D1 and D3, queue the rebuild FIRST, then an encode of the
        # same stripes into a second parity pair -- it must see the rebuilt strips
        d[:, 1].zero_()
        d[:, 3].zero_()
        pq2 = torch.zeros((B, m, L), dtype=torch.uint8, device=DEV)
        torch.cuda.synchronize()
        for s in range(B):
            ctx.reconstruct_sg(k, m, runs(d, s, n), L, [1, 3])
        for s in range(B):
            lists = runs(d, s, k) + [[(pq2[s, j].data_ptr(), L)] for j in range(m)]
            ctx.encode_sg(k, m, lists, L)
        ctx.flush()
        ctx.synchronize()
        assert (d.cpu().numpy() == ref).all()
        assert (pq2.cpu().numpy() == ref[:, k:]).all(), "encode ran before the reconstruct"
    finally:
        ctx.close()


def test_failed_flush_keeps_exactly_the_unlaunched_segments(ec):
    k, m, L, B = 16, 2, 256, 15000
    n = k + m
    row = (8 + 4 * n + 7) // 8 * 8                 # a compact row: base pointer + int32 offsets
    piece = max(4096, (1 << 20) // (row + 12))     # segments per ~1 MiB descriptor piece
    assert piece < B < 2 * piece                   # two pieces
    a, ref = stripes(k, m, L, B, 2)
    d = torch.from_numpy(a).to(DEV)
    torch.cuda.synchronize()
    ctx = ec.Ctx()
    try:
        for s in range(B):
            ctx.encode_sg(k, m, runs(d, s, n), L)
        assert ctx.queued() == B
        ctx.test_fail_after(2)           # the second piece fails before it launches
        rc = ec.lib().draid_ec_ctx_flush(ctx.h)
        assert rc < 0 and "injected" in ec.last_error()
        ctx.synchronize()
        left = ctx.queued()
        assert left == B - piece         # the first piece ran, the rest is queued
        got = d.cpu().numpy()
        done = (got[:, k] == ref[:, k]).all(axis=1)
        assert done.sum() == B - left and not done[B - left:].any() and done[:B - left].all()
        # flushing again runs the rest, nothing twice, nothing lost
        ctx.flush()
        ctx.synchronize()
        assert ctx.queued() == 0
        assert (d.cpu().numpy() == ref).all()
    finally:
        ctx.close()


def test_failed_flush_leaves_later_groups_queued(ec):
    k, m, L, B = 4, 2, 2048, 6
    n = k + m
    a, ref = stripes(k, m, L, B, 3)
    d = torch.from_numpy(a).to(DEV)
    ctx = ec.Ctx()
    try:
        torch.cuda.synchronize()
        for s in range(B):
            ctx.encode_sg(k, m, runs(d, s, n), L)
        pq2 = torch.zeros((B, 1, L), dtype=torch.uint8, device=DEV)
        torch.cuda.synchronize()
        for s in range(B):  # a second group (m = 1) behind the first
            ctx.encode_sg(k, 1, runs(d, s, k) + [[(pq2[s, 0].data_ptr(), L)]], L)
        ctx.test_fail_after(1)
        assert ec.lib().draid_ec_ctx_flush(ctx.h) < 0
        assert ctx.queued() == 2 * B       # nothing launched, everything still queued
        ctx.flush()
        ctx.synchronize()
        assert (d.cpu().numpy() == ref).all()
        assert (pq2[:, 0].cpu().numpy() == ref[:, k]).all()
    finally:
        ctx.close()


def test_tickets_complete_per_flush(ec):
    k, m, L, B = 8, 2, 65536, 64
    n = k + m
    a, ref = stripes(k, m, L, B, 4)
    d = torch.from_numpy(a).to(DEV)
    torch.cuda.synchronize()
    ctx = ec.Ctx()
    try:
        tickets = []
        for lo in range(0, B, 16):
            for s in range(lo, lo + 16):
                ctx.encode_sg(k, m, runs(d, s, n), L)
            tickets.append(ctx.flush_ticket())
        assert tickets == sorted(tickets) and len(set(tickets)) == 4
        import time
        t0 = time.time()
        while ctx.ticket_query(tickets[-1]) == 1:
            assert time.time() - t0 < 30
        for t in tickets:                      # stream order: all earlier ones are done too
            assert ctx.ticket_query(t) == 0
        assert (d.cpu().numpy() == ref).all()
        assert ec.lib().draid_ec_ctx_ticket_query(ctx.h, tickets[-1] + 1) == 1  # not issued yet
        assert "ticket" in ec.last_error()
        # more flushes than event slots: old tickets stay answerable
        for i in range(70):
            ctx.encode_sg(k, m, runs(d, i % B, n), L)
            tickets.append(ctx.flush_ticket())
        ctx.synchronize()
        assert all(ctx.ticket_query(t) == 0 for t in tickets)
    finally:
        ctx.close()


def test_context_resolves_host_pointers_of_pinned_memory(ec):
    """An SPDK buffer is a host address: with set_host_pointers the context maps
    each iovec to its device address itself, and rejects pageable memory."""
    k, m, L, B = 4, 2, 8192, 4
    n = k + m
    a, ref = stripes(k, m, L, B, 5)
    pin = torch.from_numpy(a).clone().pin_memory()
    ctx = ec.Ctx()
    try:
        ctx.set_host_pointers(True)
        for s in range(B):
            # strips split into two adjacent iovecs: merged only if adjacent for the GPU too
            lists = [[(pin[s, j].data_ptr(), L // 2), (pin[s, j].data_ptr() + L // 2, L // 2)]
                     for j in range(n)]
            ctx.encode_sg(k, m, lists, L)
        ctx.flush()
        ctx.synchronize()
        assert (pin.numpy() == ref).all()
        pin[:, 0].zero_()
        pin[:, k].zero_()
        for s in range(B):
            ctx.reconstruct_sg(k, m, runs(pin, s, n), L, [0, k])
        ctx.flush()
        ctx.synchronize()
        assert (pin.numpy() == ref).all()
        # mixed: data in device memory, parity in pinned host memory
        d = torch.from_numpy(a).to(DEV)
        pq = torch.zeros((B, m, L), dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize()
        for s in range(B):
            ctx.encode_sg(k, m, runs(d, s, k) + [[(pq[s, j].data_ptr(), L)] for j in range(m)], L)
        ctx.flush()
        ctx.synchronize()
        assert (pq.numpy() == ref[:, k:]).all()
        # pageable memory is rejected when the stripe is queued; nothing is queued
        page = np.zeros(L, np.uint8)
        bad = runs(pin, 0, n)
        bad[2] = [(page.ctypes.data, L)]
        arrs, heads, cnts = ec.Ctx._lists(bad)
        rc = ec.lib().draid_ec_ctx_encode_sg(ctx.h, k, m, heads, cnts, None, L)
        assert rc == 1 and "pinned" in ec.last_error()
        del arrs
        assert ctx.queued() == 0
    finally:
        ctx.close()


# ---- descriptor pieces uploaded ahead of the flush ----
#
# A group of small segments uploads each ~1 MiB piece of descriptors from inside
# the queueing call that completes it; the flush then only launches those pieces.
# What must hold: the same bytes as with flush-time uploads, for uniform and mixed
# segment lengths; a rollback or discard that cuts into an uploaded piece drops it.

def _piece(k, m, reconstruct=False):
    row = (8 + 4 * (k + m) + (4 if reconstruct else 0) + 7) // 8 * 8
    return max(4096, (1 << 20) // (row + 12))


@pytest.mark.parametrize("ahead", [True, False])
def test_early_uploads_same_bytes_as_flush_time_uploads(ec, ahead, monkeypatch):
    if not ahead:
        monkeypatch.setenv("DRAID_EC_CTX_STAGE_AHEAD", "0")
    k, m, L = 8, 2, 256
    n = k + m
    piece = _piece(k, m)
    B = 2 * piece + 1500                      # two whole pieces ahead, a third at the flush
    a, ref = stripes(k, m, L, B, 11)
    d = torch.from_numpy(a).to(DEV)
    torch.cuda.synchronize()
    ctx = ec.Ctx()
    try:
        seen = 0
        for s in range(B):
            ctx.encode_sg(k, m, runs(d, s, n), L)
            seen = max(seen, ctx.test_staged())
        assert seen == (2 if ahead else 0)
        assert ctx.queued() == B
        ctx.flush()
        ctx.synchronize()
        assert ctx.test_staged() == 0 and ctx.queued() == 0
        assert (d.cpu().numpy() == ref).all()
        # mixed lengths (a work list per piece): even stripes in one run, odd ones in two halves
        d[:, 1].zero_()
        d[:, 6].zero_()
        torch.cuda.synchronize()
        h = L // 2
        seen = 0
        for s in range(B):
            if s % 2 == 0:
                ctx.reconstruct_sg(k, m, runs(d, s, n), L, [6, 1])
            else:
                for off in (0, h):
                    ctx.reconstruct_sg(k, m, [[(d[s, j].data_ptr() + off, h)] for j in range(n)],
                                       h, [1, 6])
            seen = max(seen, ctx.test_staged())
        assert seen >= (2 if ahead else 0) and (ahead or seen == 0)
        ctx.flush()
        ctx.synchronize()
        assert (d.cpu().numpy() == ref).all()
    finally:
        ctx.close()


def test_rollback_and_discard_drop_early_uploads(ec):
    k, m, L = 8, 2, 256
    n = k + m
    piece = _piece(k, m)
    B = piece + 600
    a, ref = stripes(k, m, L, B, 12)
    d = torch.from_numpy(a).to(DEV)
    torch.cuda.synchronize()
    ctx = ec.Ctx()
    try:
        # a request's mark sits inside the first piece; the piece is uploaded while the
        # request is still queueing; the request then fails and is rolled back
        for s in range(piece - 300):
            ctx.encode_sg(k, m, runs(d, s, n), L)
        ctx.mark()
        for s in range(piece - 300, piece + 100):
            ctx.encode_sg(k, m, runs(d, s, n), L)
        assert ctx.test_staged() == 1
        ctx.rollback()
        assert ctx.test_staged() == 0 and ctx.queued() == piece - 300
        # other stripes take the rolled-back rows: [piece - 300, piece) stays unencoded
        for s in range(piece, B):
            ctx.encode_sg(k, m, runs(d, s, n), L)
        assert ctx.test_staged() == 1          # (piece - 300) + 600 segments: a new first piece
        ctx.flush()
        ctx.synchronize()
        got = d.cpu().numpy()
        skipped = slice(piece - 300, piece)
        assert not got[skipped, k:].any(), "a rolled-back segment ran"
        assert (got[:piece - 300] == ref[:piece - 300]).all() and (got[piece:] == ref[piece:]).all()
        # discard: a whole uploaded piece is forgotten, nothing of it runs
        d2 = torch.from_numpy(a).to(DEV)
        torch.cuda.synchronize()
        for s in range(B):
            ctx.encode_sg(k, m, runs(d2, s, n), L)
        assert ctx.test_staged() == 1
        assert ec.lib().draid_ec_ctx_discard_queued(ctx.h) == 0
        assert ctx.test_staged() == 0 and ctx.queued() == 0
        ctx.flush()
        ctx.synchronize()
        assert not d2[:, k:].any().item(), "a discarded segment ran"
        for s in range(B):
            ctx.encode_sg(k, m, runs(d2, s, n), L)
        ctx.flush()
        ctx.synchronize()
        assert (d2.cpu().numpy() == ref).all()
    finally:
        ctx.close()


def test_early_uploads_leave_slots_for_other_groups(ec):
    """More small segments than the context may hold uploaded ahead, then a second
    group in the same flush: the flush packs what is left into the free slots."""
    k, m, L = 2, 1, 64
    n = k + m
    piece = _piece(k, m)
    B = 14 * piece + 10                          # more pieces than may wait uploaded (12)
    a, ref = stripes(k, m, L, B, 13)
    d = torch.from_numpy(a).to(DEV)
    k2, m2, L2, B2 = 4, 2, 2048, 40
    a2, ref2 = stripes(k2, m2, L2, B2, 14)
    d2 = torch.from_numpy(a2).to(DEV)
    torch.cuda.synchronize()
    ctx = ec.Ctx()
    try:
        lib, h = ec.lib(), ctx.h
        import ctypes as C
        # (queued through one reused argument block: 57k stripes in a Python loop)
        iov = (ec.IoVec * n)()
        heads = (C.c_void_p * n)(*[C.addressof(iov) + j * C.sizeof(ec.IoVec) for j in range(n)])
        cnts = (C.c_int * n)(*([1] * n))
        base = d.data_ptr()
        for j in range(n):
            iov[j].iov_len = L
        for s in range(B):
            for j in range(n):
                iov[j].iov_base = base + (s * n + j) * L
            assert lib.draid_ec_ctx_encode_sg(h, k, m, heads, cnts, None, L) == 0
        assert ctx.test_staged() == 12
        for s in range(B2):
            ctx.encode_sg(k2, m2, runs(d2, s, k2 + m2), L2)
        ctx.flush()
        ctx.synchronize()
        assert ctx.test_staged() == 0
        assert (d.cpu().numpy() == ref).all()
        assert (d2.cpu().numpy() == ref2).all()
    finally:
        ctx.close()


@pytest.mark.parametrize("ahead", [True, False])
def test_one_flush_of_more_pieces_than_ring_slots(ec, ahead, monkeypatch):
    """A context records one event per flush, behind its last piece, and its sixteen ring
    slots wait on that event before they are used again.  A single batch of eighteen pieces
    comes round to slots of its own earlier pieces: those must get their event first.
    (ahead: up to twelve of the pieces are uploaded from inside the queueing calls; not
    ahead: the flush packs all of them itself.)  Then a second batch on the same context."""
    if not ahead:
        monkeypatch.setenv("DRAID_EC_CTX_STAGE_AHEAD", "0")
    k, m, L = 20, 2, 32
    n = k + m
    piece = _piece(k, m)
    B = 17 * piece + 333
    a, ref = stripes(k, m, L, B, 23)
    d = torch.from_numpy(a).to(DEV)
    base = d.data_ptr()
    torch.cuda.synchronize()
    ctx = ec.Ctx()
    try:
        for rnd in range(2):
            if rnd:
                d[:, k:].zero_()
                torch.cuda.synchronize()
            for s in range(B):
                ctx.encode_sg(k, m, [[(base + (s * n + j) * L, L)] for j in range(n)], L)
            assert ctx.queued() == B
            if rnd == 0:
                ctx.flush()
            else:
                t = ctx.flush_ticket()
            ctx.synchronize()
            if rnd:
                assert ctx.ticket_query(t) == 0
            assert ctx.queued() == 0 and ctx.test_staged() == 0
            got = d.cpu().numpy()
            bad = np.nonzero((got != ref).any(axis=(1, 2)))[0]
            assert bad.size == 0, (rnd, bad[:8])
    finally:
        ctx.close()

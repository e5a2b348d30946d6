"""draid_pq_check_static: the allocation-free variant of draid_pq_check.

Its verdict must equal draid_pq_check's on the same stripe (good parity -> 0, a
corrupted P or Q byte -> 1), on calls in a row that share the library's static
device scratch: a wide stripe first (pointer table written in several chunks),
then a smaller one (fewer vectors, shorter strips), so stale table entries and a
stale flag from the first call would show.  The parity itself comes from the
oracle, so the check kernel is judged against the CPU restatement too.
"""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def make_stripe(k, L, seed):
    """[k+2, L] device strips whose P, Q come from the CPU oracle."""
    rng = np.random.default_rng(seed)
    s = np.zeros((1, k + 2, L), np.uint8)
    s[0, :k] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    flat = s.reshape(-1)
    assert oracle.encode_strided(flat, k, 2, L, 1, L, (k + 2) * L) == 0
    return torch.from_numpy(s[0]).to(DEV)


def both(ec, strips, L, result, stream):
    ptrs = [strips[j].data_ptr() for j in range(strips.shape[0])]
    torch.cuda.synchronize()
    want = ec.pq_check(ptrs, L)
    result.fill_(0xdeadbeef - (1 << 32))  # a stale value must not survive
    torch.cuda.synchronize()
    assert ec.pq_check_static(ptrs, L, result, stream) == 0, ec.last_error()
    ec.stream_synchronize(stream)
    torch.cuda.synchronize()
    return want, int(result.item())


def test_static_check_matches_pq_check_two_calls_in_a_row(ec):
    stream = ec.stream_create()
    result = torch.zeros(1, dtype=torch.int32, device=DEV)
    try:
        # call 1: 100 + 2 vectors (four pointer chunks), 64 KiB strips, corrupted Q
        big = make_stripe(100, 65536, 1)
        want, got = both(ec, big, 65536, result, stream)
        assert (want, got) == (0, 0)
        big[101, 65535] ^= 1
        want, got = both(ec, big, 65536, result, stream)
        assert (want, got) == (1, 1)
        # call 2, straight after a failing one: smaller stripe, good parity -- the
        # flag and the table are reused and must not carry over
        small = make_stripe(8, 4096, 2)
        want, got = both(ec, small, 4096, result, stream)
        assert (want, got) == (0, 0)
        small[8, 17] ^= 0x80     # P byte
        want, got = both(ec, small, 4096, result, stream)
        assert (want, got) == (1, 1)
        small[8, 17] ^= 0x80
        small[3, 4000] ^= 4      # a data byte: both P and Q stale
        want, got = both(ec, small, 4096, result, stream)
        assert (want, got) == (1, 1)
        # minimum shape and a zero-length stripe
        tiny = make_stripe(2, 32, 3)
        assert both(ec, tiny, 32, result, stream) == (0, 0)
        assert both(ec, tiny, 0, result, stream) == (0, 0)
        # result in pinned host memory, through its device address
        pinned = torch.zeros(16, dtype=torch.int32).pin_memory()
        dptr = ec.host_device_pointer(pinned.data_ptr())
        assert dptr is not None
        ptrs = [small[j].data_ptr() for j in range(10)]
        assert ec.pq_check_static(ptrs, 4096, dptr, stream) == 0
        ec.stream_synchronize(stream)
        assert int(pinned[0]) == 1
    finally:
        ec.stream_destroy(stream)


def test_static_check_widest_and_limits(ec):
    stream = ec.stream_create()
    result = torch.zeros(1, dtype=torch.int32, device=DEV)
    try:
        k = ec.PQ_CHECK_STATIC_MAX_VECTS - 2
        wide = make_stripe(k, 1024, 4)
        assert both(ec, wide, 1024, result, stream) == (0, 0)
        wide[k - 1, 1023] ^= 0x40
        assert both(ec, wide, 1024, result, stream) == (1, 1)
        # beyond the static table, and the isa-l argument errors: rejected, nothing runs
        L = ec.lib()
        n = ec.PQ_CHECK_STATIC_MAX_VECTS + 1
        arr = (C.c_void_p * n)(*([wide.data_ptr()] * n))
        assert L.draid_pq_check_static(n, 1024, arr, result.data_ptr(), stream) == 1
        assert "257" in ec.last_error()
        assert L.draid_pq_check_static(3, 1024, arr, result.data_ptr(), stream) == 1
        assert L.draid_pq_check_static(10, 1000, arr, result.data_ptr(), stream) == 1
        assert L.draid_pq_check_static(10, 1024, arr, None, stream) == 1
    finally:
        ec.stream_destroy(stream)


def test_static_check_resolves_its_pointers(ec):
    """Like every pointer-taking entry point, the static check resolves what it is given
    before a kernel sees it: a vector or a result word in pageable host memory returns 1
    and launches nothing (it is never a GPU fault); pinned host memory is used in place,
    passed by its HOST address."""
    stream = ec.stream_create()
    result = torch.zeros(1, dtype=torch.int32, device=DEV)
    try:
        k, L = 6, 4096
        stripe = make_stripe(k, L, 9)
        ptrs = [stripe[j].data_ptr() for j in range(k + 2)]
        # a pageable vector: rejected, the result word keeps its value
        pageable = np.zeros(L, np.uint8)
        bad = list(ptrs)
        bad[2] = pageable.ctypes.data
        result.fill_(7)
        torch.cuda.synchronize()
        assert ec.lib().draid_pq_check_static(k + 2, L, (C.c_void_p * (k + 2))(*bad),
                                              result.data_ptr(), stream) == 1
        assert "pageable" in ec.last_error()
        ec.stream_synchronize(stream)
        torch.cuda.synchronize()
        assert int(result.item()) == 7
        # a pageable result word: rejected too
        word = np.zeros(1, np.uint32)
        assert ec.lib().draid_pq_check_static(k + 2, L, (C.c_void_p * (k + 2))(*ptrs),
                                              word.ctypes.data, stream) == 1
        # pinned host memory by its host address: data strips and the result word
        host = torch.empty((k + 2, L), dtype=torch.uint8).pin_memory()
        host.copy_(stripe.cpu())
        verdict = torch.full((4,), 5, dtype=torch.int32).pin_memory()
        hptrs = [host[j].data_ptr() for j in range(k + 2)]
        assert ec.pq_check_static(hptrs, L, verdict.data_ptr(), stream) == 0, ec.last_error()
        ec.stream_synchronize(stream)
        assert int(verdict[0]) == 0 and ec.pq_check(hptrs, L) == 0
        host[k + 1, 100] ^= 2
        assert ec.pq_check_static(hptrs, L, verdict.data_ptr(), stream) == 0
        ec.stream_synchronize(stream)
        assert int(verdict[0]) == 1 and ec.pq_check(hptrs, L) == 1
    finally:
        ec.stream_destroy(stream)

"""The isa-l-shaped calls on the pointers the reference actually passes.

raid5_xor_buf (raid5.c:188-201) and raid5_xor_stripe (raid5_simple.c:141-203)
hand isa-l host memory: spdk_dma_malloc'd chunk buffers and user iovecs.  The
GPU calls must therefore accept plain host pointers -- pageable memory is staged
through the device, pinned memory is reached in place -- and must never launch a
kernel on memory the GPU cannot reach.  Every result is checked bit-exact
against the CPU oracle.  Also here: reconstructs that report the stripes they
could not rebuild instead of returning success silently.
"""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def addr(a: np.ndarray) -> int:
    return a.ctypes.data


def oracle_pq(data: np.ndarray):
    """data [k, L] -> (P, Q) from the C oracle."""
    k, L = data.shape
    s = np.zeros((1, k + 2, L), np.uint8)
    s[0, :k] = data
    assert oracle.encode_strided(s.reshape(-1), k, 2, L, 1, L, (k + 2) * L) == 0
    return s[0, k].copy(), s[0, k + 1].copy()


@pytest.mark.parametrize("k,L", [(4, 65536), (8, 4096), (14, 4096), (40, 1024 + 32),
                                 (8, 1 << 20), (6, (2 << 20) + 64)])
def test_pq_gen_on_pageable_host_memory(ec, k, L):
    """malloc'd (numpy) vectors: staged in, P and Q staged out, sources untouched.  Calls
    that stage up to 8 MiB go through a pinned host arena, larger ones (the last two
    cases: 10 and 16 MiB) through a device arena and the runtime's copies."""
    rng = np.random.default_rng(k * L)
    vec = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    p = np.full(L, 0xAA, np.uint8)
    q = np.full(L, 0x55, np.uint8)
    keep = [v.copy() for v in vec]
    for v in vec + [p, q]:
        assert ec.device_pointer(addr(v), L) is None  # really pageable
    assert ec.pq_gen([addr(v) for v in vec] + [addr(p), addr(q)], L) == 0
    wp, wq = oracle_pq(np.stack(keep))
    assert (p == wp).all() and (q == wq).all()
    assert all((a == b).all() for a, b in zip(vec, keep))
    assert ec.pq_check([addr(v) for v in vec] + [addr(p), addr(q)], L) == 0
    q[L // 2] ^= 1
    assert ec.pq_check([addr(v) for v in vec] + [addr(p), addr(q)], L) == 1


def test_xor_gen_in_place_on_pageable_memory(ec):
    """raid5_xor_buf's form: xor_gen(3, size, {from, to, to}), to ^= from."""
    rng = np.random.default_rng(3)
    for L in (512, 4096, 65536 + 7):
        frm = rng.integers(0, 256, L, dtype=np.uint8)
        to = rng.integers(0, 256, L, dtype=np.uint8)
        want = frm ^ to
        assert ec.xor_gen([addr(frm), addr(to), addr(to)], L) == 0
        assert (to == want).all()
        orig = want ^ frm  # the old contents of `to`: frm ^ orig ^ to == 0
        assert ec.xor_check([addr(frm), addr(orig), addr(to)], L) == 0


def test_pinned_host_memory_by_its_host_address(ec):
    """Pinned memory passed as the HOST pointer the caller holds: used in place
    through its device address, no staging."""
    k, L = 8, 16384
    t = torch.zeros((k + 2, L), dtype=torch.uint8).pin_memory()
    a = t.numpy()
    rng = np.random.default_rng(9)
    a[:k] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    base = t.data_ptr()
    assert ec.device_pointer(base, (k + 2) * L) is not None
    assert ec.pq_gen([base + j * L for j in range(k + 2)], L) == 0
    wp, wq = oracle_pq(a[:k])
    assert (a[k] == wp).all() and (a[k + 1] == wq).all()


def test_mixed_device_pinned_and_pageable_vectors(ec):
    """One call over all three kinds of memory, rebuilt with draid_recover."""
    k, L = 6, 8192
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, (k, L), dtype=np.uint8)
    wp, wq = oracle_pq(data)
    dev_t = [torch.from_numpy(data[j]).to(DEV) for j in range(2)]
    pin_t = [torch.from_numpy(data[j]).clone().pin_memory() for j in range(2, 4)]
    page = [data[j].copy() for j in range(4, 6)]
    p = np.zeros(L, np.uint8)
    q_t = torch.zeros(L, dtype=torch.uint8, device=DEV)
    ptrs = ([t.data_ptr() for t in dev_t] + [t.data_ptr() for t in pin_t] +
            [addr(v) for v in page] + [addr(p), q_t.data_ptr()])
    torch.cuda.synchronize()
    assert ec.pq_gen(ptrs, L) == 0
    assert (p == wp).all() and (q_t.cpu().numpy() == wq).all()
    # lose a device strip and a pageable strip, rebuild both in place
    dev_t[1].zero_()
    page[0][:] = 0
    torch.cuda.synchronize()
    assert ec.recover(k, 2, L, ptrs, [1, 4]) == 0
    assert (dev_t[1].cpu().numpy() == data[1]).all()
    assert (page[0] == data[4]).all()
    # lose a pinned strip and P
    pin_t[0].zero_()
    p[:] = 0
    assert ec.recover(k, 2, L, ptrs, [2, k]) == 0
    assert (pin_t[0].numpy() == data[2]).all() and (p == wp).all()


def test_gf_vect_mul_on_pageable_memory(ec):
    L = 4096
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, L, dtype=np.uint8)
    for c in (2, 0x1D, 0x8E, 0xFF):
        dst = np.zeros(L, np.uint8)
        tbl = ec.gf_vect_mul_init(c)
        assert ec.gf_vect_mul(L, tbl, addr(src), addr(dst)) == 0
        want = np.array([oracle.gf_mul(c, int(b)) for b in src[:256]], np.uint8)
        assert (dst[:256] == want).all()
        inplace = src.copy()
        assert ec.gf_vect_mul(L, tbl, addr(inplace), addr(inplace)) == 0
        assert (inplace == dst).all()


def test_device_pointer_lookup_and_cache(ec):
    d = torch.zeros(1 << 20, dtype=torch.uint8, device=DEV)
    base = d.data_ptr()
    assert ec.device_pointer(base, 1 << 20) == base
    assert ec.device_pointer(base + 12345, 100) == base + 12345  # served from the cached range
    host = np.zeros(4096, np.uint8)
    assert ec.device_pointer(addr(host), 4096) is None
    pin = torch.zeros(8192, dtype=torch.uint8).pin_memory()
    hp = pin.data_ptr()
    dp = ec.device_pointer(hp, 8192)
    assert dp is not None and dp == ec.host_device_pointer(hp)
    assert ec.device_pointer(hp + 100, 64) == dp + 100
    ec.lib().draid_ec_pointer_cache_flush()
    assert ec.device_pointer(hp + 100, 64) == dp + 100
    assert ec.device_pointer(0, 16) is None


def test_reconstruct_reports_unrecoverable_stripes(ec):
    """A stripe listing more failures than m (or an index outside the stripe) is
    left untouched AND counted; rebuildable stripes of the same batch are rebuilt."""
    from test_gpu_parity import Batch, dev, host, sync
    k, m, L, B = 4, 1, 4096, 5
    b = Batch(k, m, L, B)
    stream = torch.cuda.current_stream().cuda_stream
    ec.encode(b.batch(ec), stream)
    sync()
    good = host(b.strips())
    v = b.strips()
    v[1, 0].fill_(7)
    v[1, 2].fill_(7)
    v[3, 1].fill_(9)
    before = host(b.strips())
    fail = np.array([0xFF, 0xFF,   # nothing lost
                     0, 2,         # two failures, one parity: unrecoverable
                     9, 0xFF,      # index outside the stripe
                     1, 0xFF,      # rebuildable
                     0xFF, 200],   # index outside the stripe
                    np.uint8)
    counter = torch.zeros(1, dtype=torch.int32, device=DEV)
    sync()
    assert ec.reconstruct_status(b.batch(ec), dev(fail), counter, stream) == 0
    sync()
    assert int(counter.item()) == 3
    after = host(b.strips())
    assert (after[3] == good[3]).all()             # stripe 3 came back
    assert (after[[0, 1, 2, 4]] == before[[0, 1, 2, 4]]).all()  # the others untouched
    # the counter accumulates; the strided form counts the same way
    base = b.buf.data_ptr() + b.offset
    assert ec.reconstruct_strided(base, k, m, L, B, b.strip_stride, b.stripe_stride, dev(fail),
                                  stream, counter=counter) == 0
    sync()
    assert int(counter.item()) == 6
    # the plain call still succeeds silently on the same table (unchanged contract)
    assert ec.reconstruct(b.batch(ec), dev(fail), stream) == 0


def test_host_reconstruct_rejects_unrecoverable_table(ec):
    k, m, L, B = 4, 2, 4096, 3
    n = k + m
    t = torch.zeros(B * n * L, dtype=torch.uint8).pin_memory()
    a = t.numpy()
    a[:] = np.random.default_rng(2).integers(0, 256, a.size, dtype=np.uint8)
    before = a.copy()
    fail = np.array([0, 1, 0, 0xFF, 1, 7], np.uint8)  # last stripe: index 7 >= k+m
    assert ec.host_reconstruct(t, k, m, L, B, L, n * L, fail.ctypes.data) == 1
    assert "nothing was rebuilt" in ec.last_error()
    assert (a == before).all()

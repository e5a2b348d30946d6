"""GPU tests of the host-resident stripe path (draid_ec_host_*) -- stripes in
pinned host memory read in place ("mapped"), or copied in / encoded or rebuilt
in HBM / copied out ("staged", and pageable memory) -- and of the strided
device API, bit-exact against the oracle."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


MODES = {"mapped": (True, 0), "staged": (True, 1), "pageable": (False, 0)}


def _host_batch(k, m, L, B, gap, seed, pinned=True):
    n = k + m
    ss = n * (L + gap) + 64
    t = torch.zeros(B * ss, dtype=torch.uint8)
    if pinned:
        t = t.pin_memory()
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


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("k,m,L,B,gap,chunk", [(8, 2, 65536, 40, 0, 0), (4, 1, 4096, 9, 512, 2),
                                               (16, 2, 8192, 5, 0, 1), (8, 2, 1000, 13, 24, 4)])
def test_host_encode_reconstruct(ec, k, m, L, B, gap, chunk, mode):
    pinned, flags = MODES[mode]
    t, a, st, ss = _host_batch(k, m, L, B, gap, seed=L + B, pinned=pinned)
    before = _strips(a, k, m, L, B, st, ss).copy()
    assert ec.host_encode(t, k, m, L, B, st, ss, chunk, flags) == 0
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
    assert ec.host_reconstruct(t, k, m, L, B, st, ss, ftab.ctypes.data, chunk, flags) == 0
    assert (_strips(a, k, m, L, B, st, ss) == ref).all()


def test_host_flags_rejected(ec):
    t = torch.zeros(10 * 4096, dtype=torch.uint8).pin_memory()
    assert ec.host_encode(t, 8, 2, 4096, 1, 4096, 10 * 4096, 0, 2) == 1  # isa-l style nonzero
    assert "flags" in ec.last_error()


@pytest.mark.parametrize("layout", ["stripe_major_gap", "strip_major"])
@pytest.mark.parametrize("k,m,L,B", [(8, 2, 65536, 64), (4, 1, 4096 + 3, 7), (16, 2, 8192, 9)])
def test_strided_device(ec, k, m, L, B, layout):
    """draid_ec_encode_strided / draid_ec_reconstruct_strided on device memory,
    stripe-major with a gap between strips and strip-major (strip j of every
    stripe contiguous), against the oracle."""
    n = k + m
    if layout == "strip_major":
        st, ss = B * L, L
    else:
        st, ss = L + 32, n * (L + 32) + 16
    span = (B - 1) * ss + (n - 1) * st + L
    rng = np.random.default_rng(L + k + B)
    img = np.zeros(span, np.uint8)
    for s in range(B):
        for j in range(k):
            img[s * ss + j * st: s * ss + j * st + L] = rng.integers(0, 256, L, dtype=np.uint8)
    d = torch.from_numpy(img).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    assert ec.encode_strided(d, k, m, L, B, st, ss, stream) == 0
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    ref = _strips(img, k, m, L, B, st, ss).copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    assert (_strips(got, k, m, L, B, st, ss) == ref).all()
    fail = np.full((B, 2), 0xFF, np.uint8)
    for s in range(B):
        nf = 1 + (s % m)
        fail[s, :nf] = rng.choice(n, nf, replace=False)
        for j in map(int, fail[s, :nf]):
            d[s * ss + j * st: s * ss + j * st + L] = 0x5A
    fd = torch.from_numpy(fail.reshape(-1).copy()).cuda()
    assert ec.reconstruct_strided(d, k, m, L, B, st, ss, fd, stream) == 0
    torch.cuda.synchronize()
    assert (_strips(d.cpu().numpy(), k, m, L, B, st, ss) == ref).all()


def test_registered_host_memory(ec):
    """SPDK's buffers are plain host memory registered once (draid_ec_host_register,
    raid5.c:1340-1342 hugepages); kernels reach them through the device address
    draid_ec_host_device_pointer returns, which may differ from the host one."""
    import ctypes
    import mmap
    k, m, L = 6, 2, 8192
    n = k + m
    mm = mmap.mmap(-1, n * L + 4096)           # page-aligned anonymous memory
    buf = np.frombuffer(mm, dtype=np.uint8)
    base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
    assert ec.host_device_pointer(base) is None  # not registered yet
    rng = np.random.default_rng(5)
    buf[:k * L] = rng.integers(0, 256, k * L, dtype=np.uint8)
    try:
        ec.host_register(base, n * L + 4096)
    except ec.DraidError as err:
        # Some boxes' drivers refuse hipHostRegister for every kind of user memory
        # (shared or private mappings, touched or not, any flag: the plain C probe
        # tools/probe/host_register_probe.c shows "invalid argument" for all of
        # them).  Registration is then unavailable to any program on the box, and
        # only memory from the pinned allocator can be mapped (covered above).
        probe = mmap.mmap(-1, 1 << 16, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        probe[:] = b"\x01" * (1 << 16)
        paddr = ctypes.addressof(ctypes.c_char.from_buffer(probe))
        rc = ec.lib().draid_ec_host_register(paddr, 1 << 16)
        if rc == 0:
            ec.host_unregister(paddr)
            raise  # the box registers memory: the failure above is ours
        pytest.skip(f"hipHostRegister is refused for any host memory on this box ({err})")
    try:
        dev = ec.host_device_pointer(base)
        assert dev is not None
        assert ec.host_device_pointer(base + 3 * L + 17) == dev + 3 * L + 17  # interior bytes
        ref = buf[:n * L].copy().reshape(n, L)
        assert oracle.encode_strided(ref.reshape(-1), k, m, L, 1, L, n * L) == 0
        # isa-l-shaped synchronous call over the registered strips
        assert ec.pq_gen([dev + j * L for j in range(n)], L) == 0
        assert (buf[:n * L].reshape(n, L) == ref).all()
        # scatter-gather context over the same memory: rebuild two lost strips
        buf[1 * L:2 * L] = 0
        buf[k * L:(k + 1) * L] = 0
        torch.cuda.synchronize()  # torch's stream before the context's own stream
        ctx = ec.Ctx()
        ctx.reconstruct_sg(k, m, [[(dev + j * L, L)] for j in range(n)], L, [1, k])
        ctx.flush()
        ctx.synchronize()
        ctx.close()
        assert (buf[:n * L].reshape(n, L) == ref).all()
    finally:
        ec.host_unregister(base)
    del buf
    mm.close()

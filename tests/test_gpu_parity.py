"""GPU parity tests: the HIP path through the C ABI, bit-exact against the CPU
oracle and the golden fixtures.  Sizes: the oracle-checked cases finish in
seconds; the BASELINE-sized cases check size-independent properties
(encode -> erase -> reconstruct round trips, sampled stripes vs the oracle).
"""
import itertools
import os

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy()


class Batch:
    """nstripes stripes of k+m strips laid out stripe-major in one device buffer,
    with an optional gap between strips, plus the device pointer table."""

    def __init__(self, k, m, L, B, gap=0, offset=0, data=None, seed=0):
        self.k, self.m, self.L, self.B = k, m, L, B
        self.strip_stride = L + gap
        self.stripe_stride = (k + m) * self.strip_stride
        total = B * self.stripe_stride + offset + 64
        self.buf = torch.zeros(total, dtype=torch.uint8, device=DEV)
        self.offset = offset
        if data is None:
            g = torch.Generator(device=DEV)
            g.manual_seed(seed)
            view = self.view()
            view[:, :k, :L] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=DEV,
                                            generator=g)
        else:
            self.view()[:, :, :L] = dev(data)
        base = self.buf.data_ptr() + offset
        ptrs = (base + np.arange(B, dtype=np.int64)[:, None] * self.stripe_stride +
                np.arange(k + m, dtype=np.int64)[None, :] * self.strip_stride)
        self.table = torch.from_numpy(ptrs.reshape(-1)).to(DEV)

    def view(self):
        return self.buf[self.offset:self.offset + self.B * self.stripe_stride].view(
            self.B, self.k + self.m, self.strip_stride)

    def strips(self):
        return self.view()[:, :, :self.L]

    def batch(self, ec):
        return ec.make_batch(self.k, self.m, self.L, self.B, self.table)


def oracle_encode(stripes: np.ndarray, k: int, m: int) -> np.ndarray:
    """stripes: [B, k+m, L] -> copy with parity from the C oracle."""
    out = np.ascontiguousarray(stripes.copy())
    B, n, L = out.shape
    flat = out.reshape(-1)
    assert oracle.encode_strided(flat, k, m, L, B, L, n * L) == 0
    return out


def sync():
    torch.cuda.synchronize()


# ------------------------------------------------------------ isa-l shaped

def test_pq_gen_gf_vect_mul_example(ec, golden):
    """gf_vect_mul.c inputs (glibc srand(0x1234)) -> P||Q fixtures, via draid_pq_gen."""
    K, L = 14, 4096
    gm = golden["gf_vect_mul_example"]
    oracle.srand(0x1234)
    for name in gm["order"]:
        data = [oracle.rand_buffer(L) for _ in range(K)]
        bufs = [dev(d) for d in data] + [torch.zeros(L, dtype=torch.uint8, device=DEV)
                                         for _ in range(2)]
        assert ec.pq_gen(bufs, L) == 0
        pq = np.fromfile(os.path.join(golden["_dir"], gm["scenarios"][name]["pq_file"]), np.uint8)
        got = np.concatenate([host(bufs[K]), host(bufs[K + 1])])
        assert (got == pq).all(), name
        assert ec.pq_check(bufs, L) == 0
        bufs[K + 1][17] ^= 1
        assert ec.pq_check(bufs, L) == 1


def test_xor_gen_raid5_shapes(ec, golden):
    """raid5.c:188-201 in-place {from,to,to}, and raid5_simple k+1 over the
    raid5_ut_ref known-answer pattern."""
    for c in golden["raid5_ut_ref"]:
        n, bl, skb = c["n"], c["blocklen"], c["strip_kb"]
        strip = skb * 1024 // bl
        k, S = n - 1, strip * bl
        buf = oracle.ut_ref_pattern(strip * k, bl)
        ref = np.fromfile(os.path.join(golden["_dir"], c["parity_file"]), np.uint8)
        data = [dev(buf[j * S:(j + 1) * S]) for j in range(k)]
        par = torch.zeros(S, dtype=torch.uint8, device=DEV)
        assert ec.xor_gen(data + [par], S) == 0
        assert (host(par) == ref).all()
        assert ec.xor_check(data + [par], S) == 0
        acc = torch.zeros(S, dtype=torch.uint8, device=DEV)  # memset + k xor_buf passes
        for d in data:
            assert ec.xor_gen([d, acc, acc], S) == 0
        assert (host(acc) == ref).all()
        par[3] ^= 0x40
        assert ec.xor_check(data + [par], S) == 1


@pytest.mark.parametrize("L", [1, 15, 16, 17, 255, 4095, 4097, 65536 + 3])
@pytest.mark.parametrize("off", [0, 1, 8])
def test_xor_gen_ragged_and_unaligned(ec, L, off):
    rng = np.random.default_rng(L + off)
    k = 5
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    big = torch.zeros((k + 1) * (L + 64) + 64, dtype=torch.uint8, device=DEV)
    views = [big[off + j * (L + 64): off + j * (L + 64) + L] for j in range(k + 1)]
    for j in range(k):
        views[j].copy_(dev(data[j]))
    assert ec.xor_gen(views, L) == 0
    ref = np.zeros(L, np.uint8)
    assert oracle.xor_gen(data + [ref], L) == 0
    assert (host(views[k]) == ref).all()
    # bytes around the destination are untouched
    assert host(big[off + k * (L + 64) + L: off + k * (L + 64) + L + 64]).sum() == 0


def test_isal_argument_rejection(ec):
    t = [torch.zeros(64, dtype=torch.uint8, device=DEV) for _ in range(4)]
    assert ec.xor_gen(t[:2], 64) == 1
    assert ec.pq_gen(t[:3], 64) == 1
    assert ec.pq_gen(t, 48) == 1
    assert ec.gf_vect_mul(40, ec.gf_vect_mul_init(3), t[0], t[1]) == 1
    assert ec.recover(2, 2, 64, t, [0, 0]) == 1
    assert ec.recover(2, 2, 64, t, [0, 4]) == 1


def test_gf_vect_mul_every_constant(ec):
    L = 4096 + 32
    rng = np.random.default_rng(7)
    src_np = rng.integers(0, 256, L, dtype=np.uint8)
    src_np[:256] = np.arange(256)
    src = dev(src_np)
    dst = torch.zeros(L, dtype=torch.uint8, device=DEV)
    ref = np.zeros(L, np.uint8)
    for c in range(256):
        tbl = ec.gf_vect_mul_init(c)
        assert ec.gf_vect_mul(L, tbl, src, dst) == 0
        assert oracle.gf_vect_mul(L, np.frombuffer(tbl, np.uint8).copy(), src_np, ref) == 0
        assert (host(dst) == ref).all(), c
    # unaligned source/destination
    s2 = torch.zeros(L + 8, dtype=torch.uint8, device=DEV)
    s2[3:3 + L].copy_(src)
    d2 = torch.zeros(L + 8, dtype=torch.uint8, device=DEV)
    assert ec.gf_vect_mul(L, ec.gf_vect_mul_init(0x8E), s2[3:3 + L], d2[5:5 + L]) == 0
    oracle.gf_vect_mul(L, oracle.gf_vect_mul_init(0x8E), src_np, ref)
    assert (host(d2[5:5 + L]) == ref).all()


@pytest.mark.parametrize("L", [32, 4096 + 32, 3 * 4096 + 96, (1 << 20) + 64])
def test_gf_vect_mul_any_table_any_length(ec, L):
    """A table from gf_vect_mul_init is a linear map and takes the 3-bit-table kernel;
    32 arbitrary bytes are not and must keep isa-l's two nibble lookups.  Lengths
    below, across and far beyond one workgroup's share (multiples of 32, isa-l's
    contract), from an unaligned address too."""
    rng = np.random.default_rng(L)
    src_np = rng.integers(0, 256, L, dtype=np.uint8)
    src = dev(src_np)
    ref = np.zeros(L, np.uint8)
    tables = [np.frombuffer(ec.gf_vect_mul_init(0xA7), np.uint8).copy(),
              rng.integers(0, 256, 32, dtype=np.uint8)]
    almost = tables[0].copy()
    almost[16 + 11] ^= 0x40          # linear but for one entry of the high half
    tables.append(almost)
    for tbl in tables:
        dst = torch.full((L + 64,), 0xEE, dtype=torch.uint8, device=DEV)
        assert ec.gf_vect_mul(L, tbl.tobytes(), src, dst[:L]) == 0
        assert oracle.gf_vect_mul(L, tbl.copy(), src_np, ref) == 0
        got = host(dst)
        assert (got[:L] == ref).all()
        assert (got[L:] == 0xEE).all()   # nothing written past the end
        dst.fill_(0xEE)
        assert ec.gf_vect_mul(L, tbl.tobytes(), src, dst[7:7 + L]) == 0
        got = host(dst)
        assert (got[7:7 + L] == ref).all()
        assert (got[:7] == 0xEE).all() and (got[7 + L:] == 0xEE).all()


@pytest.mark.parametrize("k,m", [(2, 1), (4, 1), (8, 1), (16, 1), (8, 2), (9, 2), (10, 2), (12, 2), (14, 2),
                                 (16, 2), (18, 2), (20, 1), (40, 2), (24, 2), (31, 2), (32, 2),
                                 (32, 1), (29, 1)])
def test_recover_every_failure_set(ec, k, m):
    L = 4096
    rng = np.random.default_rng(k)
    data = np.zeros((k + m, L), np.uint8)
    data[:k] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    ref = oracle_encode(data[None], k, m)[0]
    bufs = [dev(data[j]) for j in range(k + m)]
    rc = ec.xor_gen(bufs, L) if m == 1 else ec.pq_gen(bufs, L)
    assert rc == 0
    assert all((host(bufs[j]) == ref[j]).all() for j in range(k + m))
    sets = [f for nf in range(1, m + 1) for f in itertools.combinations(range(k + m), nf)]
    if len(sets) > 200:
        sets = sets[:: max(1, len(sets) // 200)] + [(0, 1), (k - 2, k - 1), (0, k), (k - 1, k + 1),
                                                    (k, k + 1)]
    for fail in sets:
        for f in fail:
            bufs[f].fill_(0xA5)
        assert ec.recover(k, m, L, bufs, list(fail)) == 0
        for j in range(k + m):
            assert (host(bufs[j]) == ref[j]).all(), (fail, j)


def test_maximum_stripe_width(ec):
    """The widest stripes the ABI accepts: encode with k = 255 data strips (Q
    coefficients up to 2^254, pointers through the device scratch table), and
    reconstruct with k + m = 255 (failure indices are bytes, 0xFF = none) at the
    ends of the coefficient range, against the oracle; wider reconstructs are
    rejected."""
    L = 512 + 32
    k, m = 255, 2
    rng = np.random.default_rng(255)
    data = np.zeros((k + m, L), np.uint8)
    data[:k] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    ref = oracle_encode(data[None], k, m)[0]
    bufs = [dev(data[j]) for j in range(k + m)]
    assert ec.pq_gen(bufs, L) == 0
    assert all((host(bufs[j]) == ref[j]).all() for j in range(k + m))
    assert ec.recover(k, m, L, bufs, [0]) == 1          # k + m = 257 > 255
    assert ec.recover(254, 2, L, bufs[:256], [0]) == 1  # 256 > 255
    k, m = 253, 2
    rng = np.random.default_rng(255)
    data = np.zeros((k + m, L), np.uint8)
    data[:k] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    ref = oracle_encode(data[None], k, m)[0]
    bufs = [dev(data[j]) for j in range(k + m)]
    assert ec.pq_gen(bufs, L) == 0
    assert all((host(bufs[j]) == ref[j]).all() for j in range(k + m))
    for fail in [(0,), (k - 1,), (0, k - 1), (k - 2, k - 1), (k - 1, k), (0, k + 1), (k, k + 1),
                 (127, 128)]:
        for f in fail:
            bufs[f].fill_(0x3C)
        assert ec.recover(k, m, L, bufs, list(fail)) == 0
        for j in range(k + m):
            assert (host(bufs[j]) == ref[j]).all(), (fail, j)


def test_gigabyte_strips_roundtrip(ec):
    """Strips of 1 GiB + 48 bytes (the 32-bit in-kernel offsets near their range,
    plus the byte tail) through the batched API: encode, erase two data strips,
    reconstruct, compare; P checked against an XOR on the device."""
    k, m, L = 2, 2, (1 << 30) + 48
    n = k + m
    buf = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    view = buf.view(n, L)
    view[:k] = torch.randint(0, 256, (k, L), dtype=torch.uint8, device=DEV, generator=g)
    table = torch.tensor([buf.data_ptr() + j * L for j in range(n)], dtype=torch.int64, device=DEV)
    batch = ec.make_batch(k, m, L, 1, table)
    sh = torch.cuda.current_stream().cuda_stream
    assert ec.encode(batch, sh) == 0
    sync()
    assert torch.equal(view[2], view[0] ^ view[1])
    good = view[:k].clone()
    view[:k] = 0
    fail = torch.tensor([0, 1], dtype=torch.uint8, device=DEV)
    assert ec.reconstruct(batch, fail, sh) == 0
    sync()
    assert torch.equal(view[:k], good)


# ------------------------------------------------------------ batched API

CONFIGS = [  # (k, m, strip bytes, stripes) -- BASELINE.json configs at reduced batch
    (4, 1, 65536, 64),
    (8, 2, 65536, 64),
    (8, 2, 131072, 32),
    (16, 2, 262144, 16),
    (14, 2, 4096, 33),
    (11, 2, 4096 + 48, 7),   # odd width, ragged length
    (21, 2, 4096 + 48, 7),   # an odd wide width (shared items, ragged last wave)
    (24, 1, 2048, 9),
    (37, 2, 4096 + 48, 7),   # run-time width: four full blocks of 8 strips and a ragged top block
    (40, 1, 2048, 9),        # run-time width, whole blocks only
    (33, 2, 1024 + 7, 5),    # run-time width, five blocks, byte tail
    (32, 2, 2048 + 16, 6),   # the widest unrolled width (two-word failure mask)
    (27, 1, 1024 + 5, 4),
    (6, 1, 1000, 5),         # ragged length, odd size
]


@pytest.mark.parametrize("k,m,L,B", CONFIGS)
def test_batched_encode_vs_oracle(ec, k, m, L, B):
    b = Batch(k, m, L, B, gap=256, seed=k * 1000 + L)
    before = host(b.strips())
    assert ec.encode(b.batch(ec), torch.cuda.current_stream().cuda_stream) == 0
    sync()
    got = host(b.strips())
    ref = oracle_encode(before, k, m)
    assert (got == ref).all()
    assert (host(b.view()[:, :, L:]) == 0).all()  # gaps untouched


def _random_failures(rng, B, k, m):
    f = np.full((B, 2), 0xFF, np.uint8)
    for s in range(B):
        kind = rng.integers(0, 6)
        if m == 1 or kind == 0:
            f[s, 0] = rng.integers(0, k + m)
        elif kind <= 2:
            f[s] = rng.choice(k, 2, replace=False)
        elif kind == 3:
            f[s] = [rng.integers(0, k), k]
        elif kind == 4:
            f[s] = [k + 1, rng.integers(0, k)]
        else:
            f[s] = [k, k + 1]
    return f


@pytest.mark.parametrize("k,m,L,B", CONFIGS)
def test_batched_reconstruct_vs_oracle(ec, k, m, L, B):
    rng = np.random.default_rng(B + k)
    b = Batch(k, m, L, B, seed=L + k)
    stream = torch.cuda.current_stream().cuda_stream
    assert ec.encode(b.batch(ec), stream) == 0
    sync()
    good = host(b.strips())
    fail = _random_failures(rng, B, k, m)
    v = b.strips()
    for s in range(B):
        for f in fail[s]:
            if f != 0xFF:
                v[s, int(f)].fill_(0x3C)
    erased = host(b.strips())
    # the oracle regenerates the same strips from the same erased stripes
    ref = erased.copy()
    assert oracle.recover_strided(ref.reshape(-1), k, m, L, B, L, (k + m) * L, fail.reshape(-1)) == 0
    assert (ref == good).all()
    assert ec.reconstruct(b.batch(ec), dev(fail.reshape(-1)), stream) == 0
    sync()
    assert (host(b.strips()) == good).all()


def test_reconstruct_ignores_unrecoverable(ec):
    k, m, L, B = 4, 1, 4096, 3
    b = Batch(k, m, L, B)
    stream = torch.cuda.current_stream().cuda_stream
    ec.encode(b.batch(ec), stream)
    sync()
    v = b.strips()
    v[1, 0].fill_(7)
    v[1, 2].fill_(7)
    before = host(b.strips())
    fail = np.array([0xFF, 0xFF, 0, 2, 9, 0xFF], np.uint8)  # none, too many, out of range
    assert ec.reconstruct(b.batch(ec), dev(fail), stream) == 0
    sync()
    assert (host(b.strips()) == before).all()


@pytest.mark.parametrize("m", [1, 2])
def test_single_data_strip_and_odd_failure_entries(ec, m):
    """k = 1 (P and Q are copies of D0), and failure tables with a duplicated index and
    the real index in the second slot: each stripe rebuilds exactly its one lost strip.
    A stripe with an out-of-range entry beside a real one is counted as unrecoverable and
    left untouched, like every counted stripe: the valid index is NOT rebuilt (a table
    with a wild entry is not to be trusted for its other one)."""
    for k, L, B in [(1, 4096 + 5, 4), (6, 2048, 5), (9, 1024, 5)]:
        n = k + m
        rng = np.random.default_rng(k + 10 * m)
        data = np.zeros((B, n, L), np.uint8)
        data[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
        ref = oracle_encode(data, k, m)
        b = Batch(k, m, L, B, data=data)
        stream = torch.cuda.current_stream().cuda_stream
        assert ec.encode(b.batch(ec), stream) == 0
        sync()
        assert (host(b.strips()) == ref).all()
        if k == 1:
            assert (ref[:, 1] == ref[:, 0]).all()        # P = D0
            if m == 2:
                assert (ref[:, 2] == ref[:, 0]).all()    # Q = 2^0 D0
        lost = [0, k, 0, n - 1, k - 1]
        rows = [[lost[0], lost[0]], [lost[1], 200], [0xFF, lost[2]], [n + 3, lost[3]],
                [lost[4], 0xFF]][:B]
        wild = [s for s in range(B) if any(e != 0xFF and e >= n for e in rows[s])]
        v = b.strips()
        for s in range(B):
            v[s, lost[s]].fill_(0xE1)
        want = ref.copy()
        for s in wild:
            want[s, lost[s]] = 0xE1                      # untouched
        fail = np.array(rows, np.uint8).reshape(-1)
        counter = torch.zeros(1, dtype=torch.int32, device=DEV)
        assert ec.reconstruct_status(b.batch(ec), dev(fail), counter, stream) == 0
        sync()
        assert (host(b.strips()) == want).all(), (k, m)
        assert int(counter.item()) == len(wild) == 2


def test_unaligned_batch(ec):
    k, m, L, B = 8, 2, 4096 + 5, 4
    b = Batch(k, m, L, B, gap=3, offset=1)
    before = host(b.strips())
    stream = torch.cuda.current_stream().cuda_stream
    assert ec.encode(b.batch(ec), stream) == 0
    sync()
    assert (host(b.strips()) == oracle_encode(before, k, m)).all()
    good = host(b.strips())
    fail = np.array([[1, 6], [0, k], [k + 1, 3], [2, 0xFF]], np.uint8)
    for s in range(B):
        for f in fail[s]:
            if f != 0xFF:
                b.strips()[s, int(f)].fill_(0)
    assert ec.reconstruct(b.batch(ec), dev(fail.reshape(-1)), stream) == 0
    sync()
    assert (host(b.strips()) == good).all()


def test_stream_api(ec):
    k, m, L, B = 8, 2, 65536, 512
    b = Batch(k, m, L, B)
    s = ec.stream_create()
    try:
        torch.cuda.synchronize()
        assert ec.encode(b.batch(ec), s) == 0
        assert ec.stream_query(s) in (0, 1)
        ec.stream_synchronize(s)
        assert ec.stream_query(s) == 0
    finally:
        ec.stream_destroy(s)
    idx = [0, 77, 511]
    got = host(b.strips()[idx])
    ref = oracle_encode(got, k, m)
    assert (got == ref).all()


# ------------------------------------------------------------ BASELINE sizes

@pytest.mark.parametrize("k,m,L,B", [(4, 1, 65536, 4096), (8, 2, 65536, 4096),
                                     (8, 2, 131072, 4096), (16, 2, 262144, 1024)])
def test_full_size_roundtrip(ec, k, m, L, B):
    """Encode the BASELINE-sized batch, check sampled stripes against the oracle,
    erase per-stripe failures, reconstruct, and require the original bytes back."""
    rng = np.random.default_rng(L + k)
    b = Batch(k, m, L, B, seed=99)
    stream = torch.cuda.current_stream().cuda_stream
    assert ec.encode(b.batch(ec), stream) == 0
    sync()
    sample = sorted(set(rng.integers(0, B, 24).tolist()) | {0, B - 1})
    got = host(b.strips()[sample])
    assert (got == oracle_encode(got, k, m)).all()
    good = b.strips().clone()
    fail = _random_failures(rng, B, k, m)
    fd = dev(fail.reshape(-1))
    # erase on the device: overwrite each failed strip
    v = b.strips()
    for slot in range(2):
        idx = np.nonzero(fail[:, slot] != 0xFF)[0]
        si = torch.from_numpy(idx).to(DEV)
        ji = torch.from_numpy(fail[idx, slot].astype(np.int64)).to(DEV)
        v[si, ji] = 0x77
    assert ec.reconstruct(b.batch(ec), fd, stream) == 0
    sync()
    assert torch.equal(b.strips(), good)


# ------------------------------------------------------------ edge buffers

def _edge_stripes(k, m, L):
    """Edge buffers: all-0x00, all-0xFF, one set bit per stripe
    (every bit position and every data strip), and the raid5_ut_ref pattern
    (0xFF fill + 8-byte LE block index, raid5_ut_ref.c:324-330)."""
    n = k + m
    rows = [np.zeros((n, L), np.uint8)]
    full = np.zeros((n, L), np.uint8)
    full[:k] = 0xFF
    rows.append(full)
    for j in range(k):
        for bit in range(8):
            r = np.zeros((n, L), np.uint8)
            r[j, (j * 131 + bit * 17) % L] = 1 << bit
            rows.append(r)
    ut = np.zeros((n, L), np.uint8)
    ut[:k] = oracle.ut_ref_pattern(k * L // 512, 512).reshape(k, L)
    rows.append(ut)
    return np.stack(rows)


@pytest.mark.parametrize("k,m", [(4, 1), (8, 2), (16, 2)])
def test_edge_buffers(ec, k, m):
    L = 4096
    data = _edge_stripes(k, m, L)
    B = data.shape[0]
    ref = oracle_encode(data, k, m)
    if m == 2:  # all-0xFF: P = 0xFF iff k odd; Q = xor of 2^j * 0xFF
        assert (ref[1, k] == (0xFF if k % 2 else 0)).all()
    b = Batch(k, m, L, B, data=data)
    stream = torch.cuda.current_stream().cuda_stream
    assert ec.encode(b.batch(ec), stream) == 0
    sync()
    assert (host(b.strips()) == ref).all()
    # every failure pair, cycled over the edge stripes
    n = k + m
    pairs = [(x, 0xFF) for x in range(n)]
    if m == 2:
        pairs += [(x, y) for x in range(n) for y in range(x + 1, n)]
    for p0 in range(0, len(pairs), B):
        fail = np.array([pairs[(p0 + s) % len(pairs)] for s in range(B)], np.uint8)
        v = b.strips()
        for s in range(B):
            for f in fail[s]:
                if f != 0xFF:
                    v[s, int(f)].fill_(0xA5)
        assert ec.reconstruct(b.batch(ec), dev(fail.reshape(-1)), stream) == 0
        sync()
        assert (host(b.strips()) == ref).all()


@pytest.mark.parametrize("k,m,L,B", [(8, 2, 65536, 4096), (16, 2, 262144, 512)])
def test_full_size_linearity(ec, k, m, L, B):
    """Parity is GF(2)-linear: encode(A ^ C) == encode(A) ^ encode(C) over the whole
    BASELINE-sized batch (a size-independent check of every stripe's P and Q)."""
    a = Batch(k, m, L, B, seed=5)
    c = Batch(k, m, L, B, seed=6)
    stream = torch.cuda.current_stream().cuda_stream
    x = Batch(k, m, L, B, data=None, seed=7)
    x.strips()[:, :k] = a.strips()[:, :k] ^ c.strips()[:, :k]
    for t in (a, c, x):
        assert ec.encode(t.batch(ec), stream) == 0
    sync()
    assert torch.equal(x.strips()[:, k:], a.strips()[:, k:] ^ c.strips()[:, k:])


# ------------------------------------------------------------ items shared by several waves

# every unrolled width: 2..4 (one wave per item; the RAID6 reconstructs of 2 and 4 with
# two vectors per lane), 5..32 with items dealt over 2 or 4 waves (21..32 have unrolled
# instances in the batched calls only; 31 and 32 with P and Q take a two-word failure
# mask)
SPLIT_K = list(range(2, 33))


@pytest.mark.parametrize("m", [1, 2])
@pytest.mark.parametrize("k", SPLIT_K)
def test_shared_items_every_length_class(ec, k, m):
    """Whole chunks, a partial last chunk of 16-byte vectors, a byte tail, and a strip
    shorter than one chunk: encode against the oracle, then every failure class
    rebuilt, with the failure table at each alignment of its first byte (the kernel
    reads it through aligned words)."""
    stream = torch.cuda.current_stream().cuda_stream
    for L, B in [(3 * 1024, 9), (2 * 1024 + 16 * 5, 7), (1024 + 16 * 3 + 7, 6), (48, 5), (5, 4),
                 (5 * 1024, 3), (4 * 1024 + 16, 3)]:
        rng = np.random.default_rng(k * 131 + m * 7 + L)
        b = Batch(k, m, L, B, gap=16 + (-L) % 16, seed=k + L)   # every strip 16-byte aligned
        assert b.table[0].item() % 16 == 0 and b.strip_stride % 16 == 0
        before = host(b.strips())
        assert ec.encode(b.batch(ec), stream) == 0
        sync()
        good = host(b.strips())
        assert (good == oracle_encode(before, k, m)).all(), (k, m, L)
        assert (host(b.view()[:, :, L:]) == 0).all()
        for at in range(4):
            fail = _random_failures(rng, B, k, m)
            v = b.strips()
            for s in range(B):
                for f in fail[s]:
                    if f != 0xFF:
                        v[s, int(f)].fill_(0xA5)
            holder = torch.zeros(2 * B + 8, dtype=torch.uint8, device=DEV)
            base = (-holder.data_ptr()) % 4          # holder[base] is word aligned
            tab = holder[base + at:base + at + 2 * B]
            tab.copy_(dev(fail.reshape(-1)))
            assert tab.data_ptr() % 4 == at
            assert ec.reconstruct(b.batch(ec), tab, stream) == 0
            sync()
            assert (host(b.strips()) == good).all(), (k, m, L, at)
            assert (host(b.view()[:, :, L:]) == 0).all()


def _random_failures_vec(rng, B, k, m):
    """_random_failures without the per-stripe Python loop, for very long batches."""
    f = np.full((B, 2), 0xFF, np.uint8)
    x = rng.integers(0, k, B)
    y = (x + 1 + rng.integers(0, k - 1, B)) % k if k > 1 else x
    kind = rng.integers(0, 6, B) if m == 2 else np.zeros(B, np.int64)
    f[:, 0] = np.where(kind == 5, k, np.where(kind == 4, k + 1, x))
    if m == 1:
        f[:, 0] = rng.integers(0, k + 1, B)
        return f
    f[:, 1] = np.where(kind == 0, 0xFF,
                       np.where(kind <= 2, y, np.where(kind == 3, k, np.where(kind == 4, x, k + 1))))
    return f


@pytest.mark.parametrize("k,m,L,B", [
    (8, 2, 64, 70000), (16, 2, 32, 66000), (4, 1, 64, 66000),   # short strips: stripes share grid rows
    (8, 2, 2049, 66000),                  # three chunks per strip: one stripe per row, z > 1
    (3, 1, 16, 64 * 65535 + 77),          # 64 stripes per row and still more rows than one z slice
    (8, 2, 16, 64 * 65535 + 77),
])
def test_more_stripes_than_one_grid_row(ec, k, m, L, B):
    """The shared-item kernels index chunks and stripes through the three grid
    dimensions: stripes of short strips share an x row, and more than 65535 rows
    spill into z."""
    stream = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(B)
    b = Batch(k, m, L, B, seed=B)
    before = host(b.strips())
    assert ec.encode(b.batch(ec), stream) == 0
    sync()
    good = host(b.strips())
    assert (good == oracle_encode(before, k, m)).all()
    del before
    fail = _random_failures_vec(rng, B, k, m)
    lost = torch.from_numpy(fail.astype(np.int64)).to(DEV)
    v = b.strips()
    rows = torch.arange(B, device=DEV)
    for t in range(2):
        sel = lost[:, t] != 0xFF
        v[rows[sel], lost[sel, t]] = 0x5A
    assert ec.reconstruct(b.batch(ec), dev(fail.reshape(-1)), stream) == 0
    sync()
    assert (host(b.strips()) == good).all()

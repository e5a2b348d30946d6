"""GPU tests of the scatter-gather context (draid_ec_ctx_*): the host iovec
walker (raid5_xor_iovs / raid5_xor_stripe restated) + gather-descriptor
kernels, bit-exact against the oracle on the gathered strips."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class Pool:
    """Strips scattered as random, misaligned pieces across one device buffer."""

    def __init__(self, rng, k, m, L, B, max_pieces=5, prefix=False):
        self.k, self.m, self.L, self.B = k, m, L, B
        self.layout = []  # [s][j] -> list of (offset, len); offsets[s][j] = prefix bytes
        self.offsets = []
        cur = 0
        for s in range(B):
            row, offs = [], []
            for j in range(k + m):
                pieces = []
                pre = int(rng.integers(1, 40)) if prefix else 0
                if pre:
                    pieces.append((cur, pre))
                    cur += pre + int(rng.integers(0, 9))
                npieces = int(rng.integers(1, max_pieces + 1))
                cuts = sorted(rng.choice(np.arange(1, L), size=min(npieces - 1, L - 1),
                                         replace=False).tolist()) if npieces > 1 else []
                bounds = [0] + cuts + [L]
                for a, b in zip(bounds, bounds[1:]):
                    if rng.random() < 0.15:
                        pieces.append((cur, 0))  # zero-length iovec
                    pieces.append((cur, b - a))
                    cur += (b - a) + int(rng.integers(0, 33))
                row.append(pieces)
                offs.append(pre)
            self.layout.append(row)
            self.offsets.append(offs)
        self.size = cur + 64
        self.host = np.zeros(self.size, np.uint8)

    def gather(self, buf, s, j):
        out, off = [], self.offsets[s][j]
        for o, n in self.layout[s][j]:
            out.append(buf[o:o + n])
        return np.concatenate(out)[off:off + self.L]

    def scatter(self, buf, s, j, data):
        pos, skip = 0, self.offsets[s][j]
        for o, n in self.layout[s][j]:
            for t in range(n):
                if skip:
                    skip -= 1
                    continue
                if pos < self.L:
                    buf[o + t] = data[pos]
                    pos += 1

    def strips(self, base, s):
        return [[(base + o, n) for o, n in self.layout[s][j]] for j in range(self.k + self.m)]


def _fill(pool, rng):
    for s in range(pool.B):
        for j in range(pool.k):
            for o, n in pool.layout[s][j]:
                pool.host[o:o + n] = rng.integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("k,m,L,B,prefix", [(4, 1, 4096, 6, False), (8, 2, 8192 + 48, 5, True),
                                            (16, 2, 3000, 3, False), (11, 2, 777, 4, True)])
@pytest.mark.parametrize("shuffled", [False, True])
@pytest.mark.parametrize("uploaded", [False, True])
def test_sg_encode_and_reconstruct(ec, k, m, L, B, prefix, shuffled, uploaded, monkeypatch):
    """shuffled: stripes queued out of address order and the context told to
    reorder every out-of-order group (ec_ctx.cpp address_order; by default only
    large scattered segments are) -- pointers, lengths and failure pairs must
    travel together.  uploaded: a launch this small reads its descriptors in place
    from pinned memory by default; the other way they are uploaded first, as every
    large launch's are."""
    if shuffled:
        monkeypatch.setenv("DRAID_EC_CTX_ADDRESS_ORDER", "2")  # read at ctx creation
    if uploaded:
        monkeypatch.setenv("DRAID_EC_CTX_INPLACE_LIMIT", "0")
    rng = np.random.default_rng(k * L + B)
    pool = Pool(rng, k, m, L, B, prefix=prefix)
    _fill(pool, rng)
    dbuf = torch.from_numpy(pool.host.copy()).to(DEV)
    base = dbuf.data_ptr()
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    ctx = ec.Ctx()
    try:
        order = rng.permutation(B).tolist() if shuffled else list(range(B))
        if shuffled and order == sorted(order):
            order = order[::-1]
        for s in order:
            offs = pool.offsets[s] if prefix else None
            assert ctx.encode_sg(k, m, pool.strips(base, s), L, offs) == 0
        assert ctx.queued() >= B
        ctx.flush()
        ctx.synchronize()
        got = dbuf.cpu().numpy()
        ref = np.stack([np.stack([pool.gather(pool.host, s, j) for j in range(k + m)])
                        for s in range(B)])
        assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, (k + m) * L) == 0
        for s in range(B):
            for j in range(k + m):
                assert (pool.gather(got, s, j) == ref[s, j]).all(), (s, j)

        # erase random failure sets (per stripe) and rebuild them through the walker
        erased = got.copy()
        fails = []
        for s in range(B):
            nf = int(rng.integers(1, m + 1))
            f = sorted(rng.choice(k + m, nf, replace=False).tolist())
            fails.append(f)
            for j in f:
                pool.scatter(erased, s, j, np.full(L, 0x5A, np.uint8))
        dbuf.copy_(torch.from_numpy(erased))
        torch.cuda.synchronize()  # torch's stream before the context's own stream
        for s in order:
            offs = pool.offsets[s] if prefix else None
            assert ctx.reconstruct_sg(k, m, pool.strips(base, s), L, fails[s], offs) == 0
        ctx.flush()
        assert ctx.query() in (0, 1)
        ctx.synchronize()
        back = dbuf.cpu().numpy()
        for s in range(B):
            for j in range(k + m):
                assert (pool.gather(back, s, j) == ref[s, j]).all(), (s, j, fails[s])
    finally:
        ctx.close()


def test_sg_rejects_short_lists(ec):
    ctx = ec.Ctx()
    try:
        t = torch.zeros(1 << 16, dtype=torch.uint8, device=DEV)
        p = t.data_ptr()
        strips = [[(p + 4096 * j, 4096)] for j in range(5)]
        strips[2] = [(p + 8192, 1000)]           # shorter than len
        before = ctx.queued()
        assert ctx.encode_sg(4, 1, strips, 4096) == 1
        assert ctx.queued() == before             # nothing queued for a rejected stripe
        assert ctx.reconstruct_sg(4, 1, [[(p, 4096)]] * 5, 4096, [0, 1]) == 1  # nfail > m
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()


def test_sg_many_stripes_one_flush(ec):
    """A whole batch of single-iovec stripes in one flush (the SPDK poller shape),
    queued out of address order over 160 MiB: the default context reorders it."""
    k, m, L, B = 8, 2, 65536, 256
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    buf = torch.randint(0, 256, (B, k + m, L), dtype=torch.uint8, device=DEV, generator=g)
    buf[:, k:] = 0
    base = buf.data_ptr()
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    ctx = ec.Ctx()
    try:
        for s in np.random.default_rng(3).permutation(B).tolist():
            strips = [[(base + (s * (k + m) + j) * L, L)] for j in range(k + m)]
            assert ctx.encode_sg(k, m, strips, L) == 0
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()
    sample = list(range(0, B, 7)) + [B - 1]
    got = buf[sample].cpu().numpy()
    ref = got.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, len(sample), L, (k + m) * L) == 0
    assert (got == ref).all()


@pytest.mark.parametrize("L,piece", [(65536, 65536), (65536, 4096), (1000, 1000), (8240, 4120)])
def test_sg_uniform_segments(ec, L, piece):
    """Every queued run the same length -> the flush sends no work list (items are
    derived in the kernel).  Encode, then dual / data+P / single reconstruct of
    erased strips, all through one context, against the oracle."""
    k, m, B = 8, 2, 64
    n = k + m
    g = torch.Generator(device=DEV)
    g.manual_seed(L + piece)
    buf = torch.randint(0, 256, (B, n, L), dtype=torch.uint8, device=DEV, generator=g)
    buf[:, k:] = 0
    base = buf.data_ptr()
    torch.cuda.synchronize()  # torch's stream before the context's own stream

    def strips(s):
        return [[(base + (s * n + j) * L + o, min(piece, L - o)) for o in range(0, L, piece)]
                for j in range(n)]

    torch.cuda.synchronize()  # torch's stream before the context's own stream
    ctx = ec.Ctx()
    try:
        for s in range(B):
            assert ctx.encode_sg(k, m, strips(s), L) == 0
        ctx.flush()
        ctx.synchronize()
        host = buf.cpu().numpy()
        ref = host.copy()
        assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
        assert (host == ref).all()
        fails = [[s % k, (s + 5) % k] if s % 3 == 0 else [s % k, k] if s % 3 == 1 else [s % n]
                 for s in range(B)]
        for s, f in enumerate(fails):
            for j in f:
                buf[s, j] = 0xC3
        torch.cuda.synchronize()  # torch's stream before the context's own stream
        for s, f in enumerate(fails):
            assert ctx.reconstruct_sg(k, m, strips(s), L, f) == 0
        ctx.flush()
        ctx.synchronize()
        assert (buf.cpu().numpy() == ref).all()
    finally:
        ctx.close()


def test_sg_adjacent_iovecs_merge(ec):
    """Memory-contiguous iovecs (and zero-length ones between them) are walked as
    one run: a strip split into adjacent pieces queues a single segment, the same
    split with gaps between the pieces queues one per piece, and both encode the
    same parity (the oracle's)."""
    k, m, L = 4, 2, 8192
    n = k + m
    cuts = [0, 1000, 1000, 4096, 5000, L]   # includes a zero-length piece
    pieces = [(a, b - a) for a, b in zip(cuts, cuts[1:])]
    gap = 64
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    buf = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=DEV, generator=g)
    buf[k:] = 0
    # the same strips scattered: piece i of strip j at j*(L+5*gap) + a + i*gap
    sc = torch.zeros(n * (L + 5 * gap), dtype=torch.uint8, device=DEV)
    for j in range(n):
        for i, (a, ln) in enumerate(pieces):
            o = j * (L + 5 * gap) + a + i * gap
            sc[o:o + ln] = buf[j, a:a + ln]
    bb, sb = buf.data_ptr(), sc.data_ptr()
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    ctx = ec.Ctx()
    try:
        assert ctx.encode_sg(k, m, [[(bb + j * L + a, ln) for a, ln in pieces]
                                    for j in range(n)], L) == 0
        assert ctx.queued() == 1
        assert ctx.encode_sg(k, m, [[(sb + j * (L + 5 * gap) + a + i * gap, ln)
                                     for i, (a, ln) in enumerate(pieces)]
                                    for j in range(n)], L) == 0
        assert ctx.queued() == 1 + sum(1 for _, ln in pieces if ln)
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()
    got = buf.cpu().numpy()
    ref = got.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, 1, L, n * L) == 0
    assert (got == ref).all()
    scat = sc.cpu().numpy()
    for j in range(k, n):
        strip = np.concatenate([scat[j * (L + 5 * gap) + a + i * gap:][:ln]
                                for i, (a, ln) in enumerate(pieces)])
        assert (strip == ref[j]).all()


@pytest.mark.parametrize("k,m,L", [(8, 2, 65536), (4, 1, 4096 + 16), (14, 2, 999), (30, 2, 2048)])
def test_sg_single_segment_flush(ec, k, m, L):
    """One contiguous stripe per flush (the queue-depth-1 case) launches the
    single-stripe kernel with its pointers in the kernel arguments; a many-segment
    flush queued before it on the same context is ordered ahead of it."""
    n = k + m
    rng = np.random.default_rng(L + k)
    host = np.zeros((3, n, L), np.uint8)
    host[:, :k] = rng.integers(0, 256, (3, k, L), dtype=np.uint8)
    ref = host.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, 3, L, n * L) == 0
    dbuf = torch.from_numpy(host).to(DEV)
    base = dbuf.data_ptr()
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    ctx = ec.Ctx()
    try:
        # stripe 0 as two segments (a split iovec), then stripes 1 and 2 alone
        half = L // 2
        strips0 = [[(base + j * L, half), (base + j * L + half + 64 * 0, L - half)] for j in range(n)]
        ctx.encode_sg(k, m, strips0, L)
        ctx.flush()
        for s in (1, 2):
            ctx.encode_sg(k, m, [[(base + (s * n + j) * L, L)] for j in range(n)], L)
            ctx.flush()
        ctx.synchronize()
        assert (dbuf.cpu().numpy() == ref).all()
        # single-segment rebuild of the worst case the level allows
        lost = [1, k] if m == 2 else [k - 1]
        for j in lost:
            dbuf[2, j] = 0xA5
        torch.cuda.synchronize()  # torch's stream before the context's own stream
        ctx.reconstruct_sg(k, m, [[(base + (2 * n + j) * L, L)] for j in range(n)], L, lost)
        ctx.flush()
        ctx.synchronize()
        assert (dbuf.cpu().numpy() == ref).all()
    finally:
        ctx.close()


@pytest.mark.parametrize("order", ["1", "2"])
def test_sg_shuffled_multi_piece(ec, order, monkeypatch):
    """More segments than one flush piece (ec_ctx.cpp kPieceBytes), queued in a
    random order with three different lengths: the reordered pieces, their
    work lists and failure pairs all line up (order 2: reordered; 1, the
    default: small segments stay as queued)."""
    monkeypatch.setenv("DRAID_EC_CTX_ADDRESS_ORDER", order)
    k, m, C, B = 8, 2, 1024, 12000
    n = k + m
    rng = np.random.default_rng(11)
    host = np.zeros((B, n, C), np.uint8)
    host[:, :k] = rng.integers(0, 256, (B, k, C), dtype=np.uint8)
    lens = [C - 16 * (s % 3) for s in range(B)]
    buf = torch.from_numpy(host).to(DEV)
    base = buf.data_ptr()

    def strips(s):
        return [[(base + (s * n + j) * C, lens[s])] for j in range(n)]

    ref = host.copy()
    for ln in (C, C - 16, C - 32):
        sel = [s for s in range(B) if lens[s] == ln]
        sub = np.ascontiguousarray(ref[sel][:, :, :ln])
        assert oracle.encode_strided(sub.reshape(-1), k, m, ln, len(sel), ln, n * ln) == 0
        ref[sel, :, :ln] = sub
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    ctx = ec.Ctx()
    try:
        for s in rng.permutation(B).tolist():
            assert ctx.encode_sg(k, m, strips(s), lens[s]) == 0
        ctx.flush()
        ctx.synchronize()
        assert (buf.cpu().numpy() == ref).all()
        fails = [sorted(rng.choice(n, 2, replace=False).tolist()) for _ in range(B)]
        erased = ref.copy()
        for s in range(B):
            for j in fails[s]:
                erased[s, j, :lens[s]] = 0xA5
        buf.copy_(torch.from_numpy(erased))
        torch.cuda.synchronize()  # torch's stream before the context's own stream
        for s in rng.permutation(B).tolist():
            assert ctx.reconstruct_sg(k, m, strips(s), lens[s], fails[s]) == 0
        ctx.flush()
        ctx.synchronize()
        assert (buf.cpu().numpy() == ref).all()
    finally:
        ctx.close()


def test_sg_full_size_shuffled(ec):
    """The headline batch (RAID6 8+2 x 64 KiB x 4096 stripes) through the context,
    queued in a random order (reordered by the default flush): parity equal to
    the batched kernel's on the same stripes and sampled stripes equal to the
    oracle's; then a random dual failure per stripe rebuilt through the context
    returns the original bytes."""
    k, m, L, B = 8, 2, 65536, 4096
    n = k + m
    g = torch.Generator(device=DEV)
    g.manual_seed(21)
    buf = torch.randint(0, 256, (B, n, L), dtype=torch.uint8, device=DEV, generator=g)
    buf[:, k:] = 0
    ref = buf.clone()
    base, rbase = buf.data_ptr(), ref.data_ptr()
    table = (rbase + torch.arange(B * n, dtype=torch.int64, device=DEV) * L).contiguous()
    stream = torch.cuda.current_stream().cuda_stream
    assert ec.encode(ec.make_batch(k, m, L, B, table), stream) == 0
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    rng = np.random.default_rng(8)

    def strips(s):
        return [[(base + (s * n + j) * L, L)] for j in range(n)]

    ctx = ec.Ctx()
    try:
        for s in rng.permutation(B).tolist():
            assert ctx.encode_sg(k, m, strips(s), L) == 0
        ctx.flush()
        ctx.synchronize()
        assert torch.equal(buf, ref)
        sample = [0, 1234, B - 1]
        got = buf[sample].cpu().numpy()
        assert (got == oracle_encode_np(got, k, m)).all()
        fails = [sorted(rng.choice(n, 2, replace=False).tolist()) for _ in range(B)]
        f = torch.tensor(fails, dtype=torch.int64, device=DEV)
        si = torch.arange(B, device=DEV)
        buf[si, f[:, 0]] = 0x6B
        buf[si, f[:, 1]] = 0xB6
        torch.cuda.synchronize()
        for s in rng.permutation(B).tolist():
            assert ctx.reconstruct_sg(k, m, strips(s), L, fails[s]) == 0
        ctx.flush()
        ctx.synchronize()
        assert torch.equal(buf, ref)
    finally:
        ctx.close()


def oracle_encode_np(stripes, k, m):
    out = np.ascontiguousarray(stripes.copy())
    B, n, L = out.shape
    assert oracle.encode_strided(out.reshape(-1), k, m, L, B, L, n * L) == 0
    return out


def test_sg_autoflush(ec):
    """draid_ec_ctx_set_autoflush: groups launch from inside the queueing calls
    once they hold N segments (encode and reconstruct groups alike); the final
    flush launches the rest, and the results equal the oracle's."""
    k, m, L, B, N = 8, 2, 16384, 300, 64
    n = k + m
    g = torch.Generator(device=DEV)
    g.manual_seed(9)
    buf = torch.randint(0, 256, (B, n, L), dtype=torch.uint8, device=DEV, generator=g)
    buf[:, k:] = 0
    base = buf.data_ptr()
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    rng = np.random.default_rng(4)

    def strips(s):
        return [[(base + (s * n + j) * L, L)] for j in range(n)]

    ctx = ec.Ctx()
    try:
        ctx.set_autoflush(N)
        for i, s in enumerate(rng.permutation(B).tolist()):
            assert ctx.encode_sg(k, m, strips(s), L) == 0
            assert ctx.queued() == (i + 1) % N
        ctx.flush()
        ctx.synchronize()
        got = buf.cpu().numpy()
        assert (got == oracle_encode_np(got, k, m)).all()
        fails = [sorted(rng.choice(n, 2, replace=False).tolist()) for _ in range(B)]
        erased = got.copy()
        for s in range(B):
            erased[s, fails[s]] = 0x99
        buf.copy_(torch.from_numpy(erased))
        torch.cuda.synchronize()
        for s in rng.permutation(B).tolist():
            assert ctx.reconstruct_sg(k, m, strips(s), L, fails[s]) == 0
        ctx.flush()
        ctx.synchronize()
        assert (buf.cpu().numpy() == got).all()
    finally:
        ctx.close()


def test_sg_back_to_back_flushes(ec):
    """Flushes issued back to back with no synchronisation between them, the
    next batch walked while the previous one's pointer tables are still being
    copied from the context's pinned storage (ec_ctx.cpp Group: double-buffered,
    a buffer is written again only after its copies are done).  Batch sizes make
    the storage grow (one batch of 2100 stripes x 16 runs x 10 strips is past its
    first 1 MiB) between small ones; every stripe must equal the oracle's."""
    k, m, L, piece = 8, 2, 8192, 512
    n = k + m
    batches = [50, 1500, 30, 2100, 7]
    B = sum(batches)
    g = torch.Generator(device=DEV)
    g.manual_seed(21)
    buf = torch.randint(0, 256, (B, n, L), dtype=torch.uint8, device=DEV, generator=g)
    buf[:, k:] = 0
    base = buf.data_ptr()
    torch.cuda.synchronize()  # torch's stream before the context's own stream

    def strips(s):  # pieces listed in reverse address order: nothing merges
        return [[(base + (s * n + j) * L + o, piece) for o in range(L - piece, -1, -piece)]
                for j in range(n)]

    def reverse_strip(x):  # the byte order the reversed iovec lists present
        return x.reshape(x.shape[:-1] + (L // piece, piece))[..., ::-1, :].reshape(x.shape)

    ctx = ec.Ctx()
    try:
        s0 = 0
        for nb in batches:
            for s in range(s0, s0 + nb):
                assert ctx.encode_sg(k, m, strips(s), L) == 0
            ctx.flush()
            s0 += nb
        ctx.synchronize()
    finally:
        ctx.close()
    got = reverse_strip(buf.cpu().numpy())
    assert (got == oracle_encode_np(got, k, m)).all()


def test_sg_fence_orders_a_request_behind_its_own_rebuild(ec):
    """Several requests share one batch.  Request A opens the encode group; request B
    (a degraded partial write, raid5.c:743-777 with a lost strip) then queues the rebuild
    of a lost data strip and, behind a fence, an encode that reads the rebuilt strip.
    Groups launch in the order of their first segment, so without the fence B's encode
    would ride with A's, ahead of B's rebuild.  Many B's and A's interleaved; every
    parity must equal the oracle's over the true data."""
    k, m, L, B = 8, 2, 16384, 24
    n = k + m
    g = torch.Generator(device=DEV)
    g.manual_seed(77)
    buf = torch.randint(0, 256, (B, n, L), dtype=torch.uint8, device=DEV, generator=g)
    ref = buf.cpu().numpy()
    ref[:, k:] = 0
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    buf.copy_(torch.from_numpy(ref))           # consistent stripes
    lost = [(3 * s + 1) % k for s in range(B)]
    out = torch.full((B, m, L), 0xEE, dtype=torch.uint8, device=DEV)   # fresh parity per stripe
    for s in range(B):
        if s % 3:                               # B-type stripes: the lost strip starts as garbage
            buf[s, lost[s]] = 0x5A
    base, obase = buf.data_ptr(), out.data_ptr()
    torch.cuda.synchronize()

    def strips(s, parity_base):
        rows = [[(base + (s * n + j) * L, L)] for j in range(k)]
        return rows + [[(parity_base(j), L)] for j in range(m)]

    ctx = ec.Ctx()
    try:
        for s in range(B):
            ctx.mark()
            if s % 3 == 0:                      # request A: a plain encode
                ctx.encode_sg(k, m, strips(s, lambda j: obase + (s * m + j) * L), L)
                continue
            # request B: rebuild the lost strip from P and Q ...
            ctx.reconstruct_sg(k, m, strips(s, lambda j: base + (s * n + k + j) * L), L,
                               [lost[s]])
            ctx.fence()
            # ... then re-encode over it into fresh parity buffers
            ctx.encode_sg(k, m, strips(s, lambda j: obase + (s * m + j) * L), L)
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()
    assert (buf.cpu().numpy() == ref).all(), "rebuilt strips"
    assert (out.cpu().numpy() == ref[:, k:]).all(), "parity encoded behind the fence"


def test_sg_mark_and_rollback_drop_exactly_one_request(ec):
    """draid_ec_ctx_mark / rollback: a request whose later queueing call fails leaves
    nothing queued (its buffers are reused by the next owner), earlier requests stay."""
    k, m, L = 4, 2, 4096
    n = k + m
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    buf = torch.randint(0, 256, (3, n, L), dtype=torch.uint8, device=DEV, generator=g)
    buf[:, k:] = 0x11
    before = buf.cpu().numpy()
    base = buf.data_ptr()
    torch.cuda.synchronize()

    def strips(s):
        return [[(base + (s * n + j) * L, L)] for j in range(n)]

    ctx = ec.Ctx()
    try:
        assert ec.lib().draid_ec_ctx_rollback(ctx.h) == 1      # no mark yet
        ctx.encode_sg(k, m, strips(0), L)                       # request 0 stays
        ctx.mark()
        ctx.reconstruct_sg(k, m, strips(1), L, [0, 2])          # request 1: two groups ...
        ctx.fence()
        ctx.encode_sg(k, m, strips(1), L)
        assert ctx.queued() == 3
        ctx.rollback()                                          # ... all dropped
        assert ctx.queued() == 1
        ctx.mark()
        ctx.encode_sg(k, m, strips(2), L)                       # request 2 queues normally
        ctx.flush()
        assert ec.lib().draid_ec_ctx_rollback(ctx.h) == 1      # launched: cannot be undone
        ctx.synchronize()
    finally:
        ctx.close()
    got = buf.cpu().numpy()
    ref = before.copy()
    ref[:, k:] = 0
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, 3, L, n * L) == 0
    assert (got[0] == ref[0]).all() and (got[2] == ref[2]).all()
    assert (got[1] == before[1]).all(), "the rolled-back request touched its buffers"


def test_sg_rows_compact_and_wide(ec, monkeypatch):
    """The context queues a run as a compact row (base pointer + 32-bit offsets) when
    its strips lie within 2 GiB of the first one, and as a row of 64-bit pointers when
    they do not; both kinds may share a batch.  Stripes whose strips sit at both ends
    of a 2.6 GiB buffer (wide rows) are queued between ordinary ones (compact rows),
    encoded and rebuilt; then the whole batch again with compact rows switched off
    (DRAID_EC_CTX_ROWS=64), which must give the same bytes."""
    k, m, L, B = 5, 2, 4096 + 16, 12
    n = k + m
    far = (1 << 31) + (300 << 20)                     # > 2 GiB
    big = torch.zeros(far + B * n * L + 4096, dtype=torch.uint8, device=DEV)
    rng = np.random.default_rng(99)
    data = rng.integers(0, 256, (B, n, L), dtype=np.uint8)
    data[:, k:] = 0
    ref = data.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    base = big.data_ptr()

    def where(s, j):      # odd stripes: strips 1, 3, ... live 2.3 GiB above the others
        off = (s * n + j) * L
        return off + (far if (s % 2 == 1 and j % 2 == 1) else 0)

    def strips(s):
        return [[(base + where(s, j), L)] for j in range(n)]

    def put(vals):
        for s in range(B):
            for j in range(n):
                o = where(s, j)
                big[o:o + L] = torch.from_numpy(vals[s, j]).to(DEV)

    def get():
        out = np.zeros((B, n, L), np.uint8)
        for s in range(B):
            for j in range(n):
                o = where(s, j)
                out[s, j] = big[o:o + L].cpu().numpy()
        return out

    for rows in (None, "64"):
        if rows:
            monkeypatch.setenv("DRAID_EC_CTX_ROWS", rows)     # read at ctx creation
        put(data)
        torch.cuda.synchronize()
        ctx = ec.Ctx()
        try:
            for s in range(B):
                ctx.encode_sg(k, m, strips(s), L)
            assert ctx.queued() == B
            ctx.flush()
            ctx.synchronize()
            assert (get() == ref).all(), rows
            fails = [[(s + 1) % k, k + (s % 2)] for s in range(B)]   # a data strip and P or Q
            erased = ref.copy()
            for s in range(B):
                for f in fails[s]:
                    erased[s, f] = 0x3C
            put(erased)
            torch.cuda.synchronize()
            for s in range(B):
                ctx.reconstruct_sg(k, m, strips(s), L, fails[s])
            ctx.flush()
            ctx.synchronize()
            assert (get() == ref).all(), rows
        finally:
            ctx.close()

"""GPU tests of the read-modify-write parity update (draid_ec_ctx_update_sg):
after P ^= sum(delta), Q ^= sum(2^i delta) the parity must equal a full
re-encode of the updated stripe by the oracle (raid5.c:705-741 semantics,
extended to Q)."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _runs(rng, base, length, pieces):
    """Split [base, base+length) into up to `pieces` contiguous runs."""
    if pieces <= 1 or length < 2:
        return [(base, length)]
    cuts = sorted(rng.choice(np.arange(1, length), size=min(pieces - 1, length - 1),
                             replace=False).tolist())
    b = [0] + cuts + [length]
    return [(base + x, y - x) for x, y in zip(b, b[1:])]


@pytest.mark.parametrize("k,m,L,B", [(4, 1, 4096, 6), (8, 2, 65536, 5), (16, 2, 8192, 4),
                                     (8, 2, 1000, 5)])
@pytest.mark.parametrize("uploaded", [False, True])
def test_rmw_update_matches_reencode(ec, k, m, L, B, uploaded, monkeypatch):
    if uploaded:  # descriptors uploaded first instead of read in place (small launches)
        monkeypatch.setenv("DRAID_EC_CTX_INPLACE_LIMIT", "0")
    rng = np.random.default_rng(k * 100 + L)
    n = k + m
    host = np.zeros((B, n, L), np.uint8)
    host[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    assert oracle.encode_strided(host.reshape(-1), k, m, L, B, L, n * L) == 0
    stripes = torch.from_numpy(host.copy()).to(DEV)
    newdata = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).to(DEV)
    olddata = stripes[:, :k].clone()           # the RMW preread of the touched chunks
    torch.cuda.synchronize()  # torch's stream before the context's own stream
    expect = host.copy()
    ctx = ec.Ctx()
    try:
        for s in range(B):
            nd = int(rng.integers(1, k + 1))
            idx = sorted(rng.choice(k, nd, replace=False).tolist(), key=lambda _: rng.random())
            a = int(rng.integers(0, L // 2))
            b = int(rng.integers(a + 1, L + 1))
            ln = b - a
            pc = int(rng.integers(1, 4))
            old = [_runs(rng, olddata[s, i].data_ptr() + a, ln, pc) for i in idx]
            new = [_runs(rng, newdata[s, i].data_ptr() + a, ln, pc) for i in idx]
            par = [_runs(rng, stripes[s, k + j].data_ptr() + a, ln, pc) for j in range(m)]
            assert ctx.update_sg(k, m, idx, old, new, par, ln) == 0
            for i in idx:
                expect[s, i, a:b] = newdata[s, i, a:b].cpu().numpy()
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()
    ref = expect.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    got = stripes.cpu().numpy()
    assert (got[:, k:] == ref[:, k:]).all()
    assert (got[:, :k] == host[:, :k]).all()      # update touches parity only


@pytest.mark.parametrize("nd", [1, 2, 3])
@pytest.mark.parametrize("k,m", [(4, 1), (8, 2), (16, 2), (40, 2)])
def test_rmw_each_touched_count_and_exponent(ec, k, m, nd):
    """nd = 1 and 2 have kernels of their own, 3 runs the run-time loop; over the
    batch every data index (every power of two up to 2^(k-1)) multiplies a delta,
    in both orders, on whole strips (16-byte vectors plus a ragged tail)."""
    L = 4096 + 16 + 5
    B = 2 * k
    n = k + m
    rng = np.random.default_rng(7000 + 10 * k + nd)
    host = np.zeros((B, n, L), np.uint8)
    host[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    assert oracle.encode_strided(host.reshape(-1), k, m, L, B, L, n * L) == 0
    stripes = torch.from_numpy(host.copy()).to(DEV)
    newdata = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).to(DEV)
    olddata = stripes[:, :k].clone()
    torch.cuda.synchronize()
    expect = host.copy()
    ctx = ec.Ctx()
    try:
        for s in range(B):
            idx = [(s + 5 * t) % k for t in range(nd)]
            if len(set(idx)) != nd:
                idx = [(s + t) % k for t in range(nd)]
            if s >= k:
                idx = idx[::-1]
            old = [[(olddata[s, i].data_ptr(), L)] for i in idx]
            new = [[(newdata[s, i].data_ptr(), L)] for i in idx]
            par = [[(stripes[s, k + j].data_ptr(), L)] for j in range(m)]
            assert ctx.update_sg(k, m, idx, old, new, par, L) == 0
            for i in idx:
                expect[s, i] = newdata[s, i].cpu().numpy()
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()
    ref = expect.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    got = stripes.cpu().numpy()
    assert (got[:, k:] == ref[:, k:]).all()
    assert (got[:, :k] == host[:, :k]).all()


def test_rmw_rejects_bad_indices(ec):
    ctx = ec.Ctx()
    try:
        t = torch.zeros(1 << 16, dtype=torch.uint8, device=DEV)
        p = t.data_ptr()
        one = [[(p, 4096)]]
        assert ctx.update_sg(4, 1, [4], one, one, one, 4096) == 1          # index >= k
        assert ctx.update_sg(4, 1, [1, 1], one * 2, one * 2, one, 4096) == 1  # duplicate
        ctx.flush()
        ctx.synchronize()
    finally:
        ctx.close()

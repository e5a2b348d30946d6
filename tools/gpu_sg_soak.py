"""Randomised sweep of the scatter-gather context on the GPU: encode_sg, reconstruct_sg
and update_sg over random widths (compiled and run-time), lengths, misaligned iovec
splits, zero-length iovecs and prefixes, in and out of address order, against the CPU
oracle -- beyond the fixed grid of tests/test_gpu_sg.py and tests/test_gpu_rmw.py.
Exits non-zero at the first mismatch, naming the case."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import draid_ec as ec  # noqa: E402
import oracle  # noqa: E402
from test_gpu_sg import Pool, _fill  # noqa: E402

DEV = "cuda:0"
cases = int(sys.argv[1]) if len(sys.argv) > 1 else 300
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 91)


def fail(msg):
    print(msg, flush=True)
    sys.exit(1)


for c in range(cases):
    k = int(rng.integers(2, 25))
    m = int(rng.integers(1, 3))
    L = int(rng.choice([1, 16, 48, 1000, 1024, 2048 + 16, 3000])) if rng.random() < 0.6 \
        else int(rng.integers(1, 3000))
    B = int(rng.integers(1, 6))
    prefix = bool(rng.random() < 0.3)
    shuffled = bool(rng.random() < 0.5)
    case = f"case {c}: k={k} m={m} L={L} B={B} prefix={prefix} shuffled={shuffled}"
    os.environ["DRAID_EC_CTX_ADDRESS_ORDER"] = "2" if shuffled else "1"
    pool = Pool(rng, k, m, L, B, prefix=prefix)
    _fill(pool, rng)
    dbuf = torch.from_numpy(pool.host.copy()).to(DEV)
    base = dbuf.data_ptr()
    torch.cuda.synchronize()
    ctx = ec.Ctx()
    try:
        order = rng.permutation(B).tolist() if shuffled else list(range(B))
        for s in order:
            assert ctx.encode_sg(k, m, pool.strips(base, s), L,
                                 pool.offsets[s] if prefix else None) == 0, case
        ctx.flush()
        ctx.synchronize()
        got = dbuf.cpu().numpy()
        ref = np.stack([np.stack([pool.gather(pool.host, s, j) for j in range(k + m)])
                        for s in range(B)])
        assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, (k + m) * L) == 0
        for s in range(B):
            for j in range(k + m):
                if not (pool.gather(got, s, j) == ref[s, j]).all():
                    fail(f"ENCODE_SG MISMATCH {case} stripe {s} strip {j}")
        # read-modify-write of a random subset of data strips: new data in a second buffer
        if L >= 2:
            new = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).to(DEV)
            torch.cuda.synchronize()
            expect = ref.copy()
            olds = []
            for s in order:
                nd = int(rng.integers(1, k + 1))
                idx = rng.choice(k, nd, replace=False).tolist()
                old = torch.from_numpy(np.stack([ref[s, i] for i in idx])).to(DEV)
                olds.append(old)
                torch.cuda.synchronize()
                strips = pool.strips(base, s)
                if prefix:  # parity iovecs carry a prefix the update call has no offset for
                    continue
                assert ctx.update_sg(k, m, idx, [[(old[t].data_ptr(), L)] for t in range(nd)],
                                     [[(new[s, i].data_ptr(), L)] for i in idx],
                                     [strips[k + j] for j in range(m)], L) == 0, case
                for i in idx:
                    expect[s, i] = new[s, i].cpu().numpy()
            ctx.flush()
            ctx.synchronize()
            if not prefix:
                got = dbuf.cpu().numpy()
                assert oracle.encode_strided(expect.reshape(-1), k, m, L, B, L, (k + m) * L) == 0
                for s in range(B):
                    for j in range(k, k + m):
                        if not (pool.gather(got, s, j) == expect[s, j]).all():
                            fail(f"UPDATE_SG MISMATCH {case} stripe {s} parity {j - k}")
                # put the updated data in place so the stripes are consistent again
                host = got.copy()
                for s in range(B):
                    for j in range(k):
                        pool.scatter(host, s, j, expect[s, j])
                dbuf.copy_(torch.from_numpy(host))
                torch.cuda.synchronize()
                ref = expect
        # erase and rebuild
        cur = dbuf.cpu().numpy()
        fails = []
        for s in range(B):
            nf = int(rng.integers(1, m + 1))
            f = sorted(rng.choice(k + m, nf, replace=False).tolist())
            fails.append(f)
            for j in f:
                pool.scatter(cur, s, j, np.full(L, 0x5A, np.uint8))
        dbuf.copy_(torch.from_numpy(cur))
        torch.cuda.synchronize()
        for s in order:
            assert ctx.reconstruct_sg(k, m, pool.strips(base, s), L, fails[s],
                                      pool.offsets[s] if prefix else None) == 0, case
        ctx.flush()
        ctx.synchronize()
        back = dbuf.cpu().numpy()
        for s in range(B):
            for j in range(k + m):
                if not (pool.gather(back, s, j) == ref[s, j]).all():
                    fail(f"RECONSTRUCT_SG MISMATCH {case} stripe {s} strip {j} lost {fails[s]}")
    finally:
        ctx.close()
    if (c + 1) % 25 == 0:
        print(f"{c + 1} cases ok (last: {case})", flush=True)
print(f"sg soak: {cases} random cases bit-exact against the oracle")

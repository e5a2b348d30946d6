"""Multi-rank (gloo, world_size 2, CPU) tests of the stripe sharding the GPU path
uses: every stripe is owned by exactly one rank, per-rank results combine to the
single-process result, and the bench's cross-rank aggregation is max-time /
sum-units.  No collective is on the data path -- the gather below is only the
test's check."""
import hashlib
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import oracle

K, M, L, B_TOTAL = 8, 2, 4096, 37


def _stripes(lo, hi):
    rng = np.random.default_rng(1234)
    allb = rng.integers(0, 256, (B_TOTAL, K + M, L), dtype=np.uint8)
    allb[:, K:] = 0
    return np.ascontiguousarray(allb[lo:hi])


def _digest(buf):
    return [hashlib.sha256(s.tobytes()).hexdigest() for s in buf]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.shard_range(B_TOTAL, rank, world)
    buf = _stripes(lo, hi)
    assert oracle.encode_strided(buf.reshape(-1), K, M, L, hi - lo, L, (K + M) * L) == 0
    fail = bench.failure_pairs(hi - lo, K, 0x1234 ^ lo).reshape(-1)
    good = buf.copy()
    for s in range(hi - lo):
        buf[s, fail[2 * s]] = 0
        buf[s, fail[2 * s + 1]] = 0
    assert oracle.recover_strided(buf.reshape(-1), K, M, L, hi - lo, L, (K + M) * L, fail) == 0
    assert (buf == good).all()
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, _digest(buf)))
    el, units = bench.reduce_timing(1.0 + rank, 10.0 * (hi - lo), torch.device("cpu"))
    if rank == 0:
        q.put((parts, el, units))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for total in (1, 7, 4096, 16384):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = bench.shard_range(total, r, world)
                seen.extend(range(lo, hi))
            assert seen == list(range(total))


def test_c_abi_split_is_a_partition_and_agrees_with_the_bench():
    """draid_ec_shard_of / _range / _count (the split a single-process target uses,
    draid_ec_mgpu) own every stripe exactly once under both policies; the range
    policy is the bench's per-rank split."""
    import draid_ec as ec
    for total in (1, 7, 37, 4096, 16384, (1 << 40) + 3):
        for g in (1, 2, 3, 8):
            ranges = [ec.shard_range(total, g, d) for d in range(g)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            if total <= 16384:
                assert ranges == [bench.shard_range(total, d, g) for d in range(g)]
            for pol in (ec.SHARD_RANGE, ec.SHARD_MOD):
                assert sum(ec.shard_count(total, g, d, pol) for d in range(g)) == total
            probe = range(total) if total <= 4096 else [0, 1, total // 3, total // 2, total - 2,
                                                        total - 1]
            for s in probe:
                d = ec.shard_of(s, total, g, ec.SHARD_RANGE)
                assert ranges[d][0] <= s < ranges[d][1]
                assert ec.shard_of(s, total, g, ec.SHARD_MOD) == s % g
            assert ec.shard_of(total, total, g, ec.SHARD_RANGE) == -1


def _mod_worker(rank, world, port, q):
    """Rank r plays device slot r of a single-process target: it takes the stripes the
    C ABI routes to it (s mod G), encodes them, and the union is the whole volume."""
    import draid_ec as ec
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = [s for s in range(B_TOTAL) if ec.shard_of(s, B_TOTAL, world, ec.SHARD_MOD) == rank]
    assert len(mine) == ec.shard_count(B_TOTAL, world, rank, ec.SHARD_MOD)
    allb = _stripes(0, B_TOTAL)
    buf = np.ascontiguousarray(allb[mine])
    assert oracle.encode_strided(buf.reshape(-1), K, M, L, len(mine), L, (K + M) * L) == 0
    parts = [None] * world
    dist.all_gather_object(parts, (mine, _digest(buf)))
    if rank == 0:
        q.put(parts)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_with_the_mod_split_cover_the_volume():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_mod_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = _stripes(0, B_TOTAL)
    assert oracle.encode_strided(single.reshape(-1), K, M, L, B_TOTAL, L, (K + M) * L) == 0
    want = _digest(single)
    got = {}
    for mine, digests in parts:
        for s, d in zip(mine, digests):
            assert s not in got
            got[s] = d
    assert [got[s] for s in range(B_TOTAL)] == want


def test_two_rank_shards_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts, el, units = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts.sort()
    assert parts[0][0] == 0 and parts[-1][1] == B_TOTAL
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    merged = [d for p in parts for d in p[2]]
    single = _stripes(0, B_TOTAL)
    assert oracle.encode_strided(single.reshape(-1), K, M, L, B_TOTAL, L, (K + M) * L) == 0
    assert merged == _digest(single)
    assert el == 2.0                      # max over ranks
    assert units == 10.0 * B_TOTAL        # sum over ranks

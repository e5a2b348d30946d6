"""One process driving several device slots (draid_ec_mgpu): the stripes of a
volume are routed to slots with the C ABI's own split (range and s mod G), each
slot encodes and rebuilds its shard on its own stream, and the union is
bit-exact against the CPU oracle.  On a one-GPU box the slots all map to GPU 0,
which still exercises the routing, the per-slot streams and the completion
query; with more GPUs visible the slots spread over them."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("policy_name", ["range", "mod"])
@pytest.mark.parametrize("slots", [1, 2, 3])
def test_single_process_split_matches_oracle(ec, slots, policy_name):
    k, m, L, B = 8, 2, 8192, 53
    n = k + m
    policy = ec.SHARD_RANGE if policy_name == "range" else ec.SHARD_MOD
    ngpu = torch.cuda.device_count()
    devices = [d % ngpu for d in range(slots)]
    rng = np.random.default_rng(slots * 7 + policy)
    vol = np.zeros((B, n, L), np.uint8)
    vol[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    ref = vol.copy()
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    fail_all = np.stack([rng.integers(0, k, B), np.full(B, k + 1)], axis=1).astype(np.uint8)  # D + Q

    mg = ec.MultiGpu(devices)
    try:
        assert mg.n == slots
        owner = [ec.shard_of(s, B, slots, policy) for s in range(B)]
        shard, bufs, tables, batches, fails, counters = [], [], [], [], [], []
        for d in range(slots):
            mine = [s for s in range(B) if owner[s] == d]
            assert len(mine) == ec.shard_count(B, slots, d, policy)
            dev = torch.device("cuda", mg.device(d))
            buf = torch.from_numpy(np.ascontiguousarray(vol[mine])).to(dev)
            table = (buf.data_ptr() + torch.arange(len(mine) * n, dtype=torch.int64, device=dev) * L)
            shard.append(mine)
            bufs.append(buf)
            tables.append(table)
            batches.append(ec.make_batch(k, m, L, len(mine), table))
            fails.append(torch.from_numpy(np.ascontiguousarray(fail_all[mine]).reshape(-1)).to(dev))
            counters.append(torch.zeros(1, dtype=torch.int32, device=dev))
        for d in range(ngpu):
            torch.cuda.synchronize(d)
        assert mg.encode(batches) == 0
        while mg.query() == 1:
            pass
        for d in range(slots):
            assert (bufs[d].cpu().numpy() == ref[shard[d]]).all()
        # lose one data strip and Q everywhere, rebuild on every slot
        for d in range(slots):
            for i, s in enumerate(shard[d]):
                bufs[d][i, int(fail_all[s, 0])] = 0
                bufs[d][i, k + 1] = 0
        for d in range(ngpu):
            torch.cuda.synchronize(d)
        assert mg.reconstruct(batches, fails, counters) == 0
        mg.synchronize()
        assert mg.query() == 0
        for d in range(slots):
            assert (bufs[d].cpu().numpy() == ref[shard[d]]).all()
            assert int(counters[d].item()) == 0
    finally:
        mg.close()


def test_mgpu_argument_errors(ec):
    import ctypes as C
    L = ec.lib()
    h = C.c_void_p()
    bad = (C.c_int * 1)(99)
    assert L.draid_ec_mgpu_create(C.byref(h), 1, bad) == 1 and "out of range" in ec.last_error()
    assert L.draid_ec_mgpu_create(None, 1, None) == 1
    assert L.draid_ec_mgpu_query(None) == 1
    assert L.draid_ec_mgpu_encode(None, None) == 1

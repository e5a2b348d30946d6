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


def test_isal_calls_on_one_thread_across_two_gpus(ec):
    """The relinked reference calls xor_gen / pq_gen from whichever reactor thread, with
    whichever GPU that thread last selected (raid5.c:188-201 is the call site).  The calls'
    per-thread device scratch -- the staging arena for pageable vectors, the pointer table
    of wide stripes, the check flag -- is memory of ONE GPU, so it is kept per GPU: the
    same thread runs pq_gen / pq_check / recover on pageable memory on GPU 0, then on
    GPU 1, then on GPU 0 again, and a GPU 0 device pointer is refused on GPU 1 instead of
    being handed to a kernel there."""
    import ctypes as C
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs: one GPU cannot show state of GPU 0 being used on GPU 1")
    k, L = 40, 8192                      # 42 vectors: beyond kernel arguments -> pointer table
    rng = np.random.default_rng(11)
    host = np.zeros((k + 2, L), np.uint8)
    host[:k] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    ref = host.copy().reshape(1, k + 2, L)
    assert oracle.encode_strided(ref.reshape(-1), k, 2, L, 1, L, (k + 2) * L) == 0
    ptrs = [host[j].ctypes.data for j in range(k + 2)]
    lib = ec.lib()
    try:
        for dev in (0, 1, 0):
            assert lib.draid_ec_set_device(dev) == 0
            host[k:] = 0
            assert ec.pq_gen(ptrs, L) == 0                      # pageable: staged on this GPU
            assert (host == ref[0]).all(), dev
            assert ec.pq_check(ptrs, L) == 0
            host[3] ^= 0xFF
            assert ec.pq_check(ptrs, L) == 1
            host[3] = 0
            host[17] = 0
            assert ec.recover(k, 2, L, ptrs, [3, 17]) == 0
            assert (host == ref[0]).all(), dev
        # device memory of GPU 0 offered to a call running on GPU 1
        on0 = torch.from_numpy(ref[0]).to("cuda:0")
        torch.cuda.synchronize(0)
        d0 = [on0[j].data_ptr() for j in range(k + 2)]
        assert lib.draid_ec_set_device(1) == 0
        arr = (C.c_void_p * (k + 2))(*d0)
        assert lib.draid_pq_check(k + 2, L, arr) == 1
        assert "other than the current one" in ec.last_error()
        out = C.c_void_p()
        assert lib.draid_ec_device_pointer(d0[0], L, C.byref(out)) == 1
        assert lib.draid_ec_set_device(0) == 0
        assert ec.pq_check(d0, L) == 0
        assert lib.draid_ec_device_pointer(d0[0], L, C.byref(out)) == 0 and out.value == d0[0]
    finally:
        lib.draid_ec_set_device(0)

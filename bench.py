#!/usr/bin/env python3
"""bench.py -- device-resident RAID6 8+2 encode + reconstruct at 64 KiB strips.

Metric (BASELINE.json): "GiB/s device-resident RAID6 8+2 encode+reconstruct,
64KiB strips, 1/2/4/8 GPU".

One step = one pass of the hot path over one batch resident in HBM:
  1. full-stripe P+Q encode of every stripe             (draid_ec_encode)
  2. dual-data-failure reconstruct of every stripe      (draid_ec_reconstruct)
     -- two data strips per stripe (x != y drawn from a seeded RNG) are
     regenerated from the 6 surviving data strips + P + Q.
Both go through the C ABI of libdraid_ec.so on the stream the events time.

value = user-data bytes through both passes, 2 * k * S * B per GPU, summed over
ranks, / max-over-ranks wall time, in GiB/s.  Stripes shard across ranks by
index (weak scaling: B stripes per GPU), no collective on the data path; the
only collectives are the contract's barrier and the max/sum of the timings.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE env).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def shard_range(nstripes_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous stripe range [lo, hi) of a rank."""
    return nstripes_total * rank // world, nstripes_total * (rank + 1) // world


def reduce_timing(elapsed: float, units: float, device) -> tuple[float, float]:
    """Contract aggregation across ranks: max of the wall times, sum of the units."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed, units
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    u = torch.tensor([units], dtype=torch.float64, device=device)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), float(u.item())


def failure_pairs(nstripes: int, k: int, seed: int) -> np.ndarray:
    """[nstripes, 2] distinct lost data indices per stripe (dual data failure)."""
    rng = np.random.default_rng(seed)
    x = rng.integers(0, k, nstripes)
    y = (x + rng.integers(1, k, nstripes)) % k
    return np.stack([x, y], axis=1).astype(np.uint8)


def load_pmc_traffic(workload: str):
    """HBM bytes per encode launch from the committed rocprofv3 PMC summary
    (profiles/pmc_<workload>.json, written by tools/collect_pmc.py), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("encode_hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def cpu_baseline(k: int, m: int, S: int, seconds: float, threads: int) -> dict:
    """The C oracle (isa-l v2.30 restatement, oracle/) timed on the host cores on
    a bounded sample of the same workload: 64 stripes, encode + dual reconstruct."""
    import oracle
    B = 64
    buf = np.frombuffer(np.random.default_rng(1).bytes((k + m) * S * B), np.uint8).copy()
    fail = failure_pairs(B, k, 7).reshape(-1)
    el, passes = oracle.bench_encode_reconstruct(buf, k, m, S, B, S, (k + m) * S, fail, True,
                                                 threads, seconds)
    if el <= 0:
        return {"value": None, "error": "oracle bench failed"}
    user = 2.0 * k * S * B * passes
    return {"value": round(user / el / GIB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{B} stripes x RAID6 {k}+{m} x {S // 1024} KiB, encode + dual-data "
                      f"reconstruct, {passes} passes in {el:.1f}s, C oracle (64-bit SWAR "
                      f"restatement of isa-l pq_gen_base + nibble-table gf_vect_mul), "
                      f"-O3 -mavx2, {threads} pthreads"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--strip-kib", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--variant", type=int, default=0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import draid_ec as ec

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ec.lib()
    ec.set_variant(args.variant)

    k, m, S, B = args.k, 2, args.strip_kib * 1024, args.stripes
    n = k + m
    # Stripe-major layout in HBM: stripe s = [D0 .. D{k-1} P Q], strips contiguous.
    buf = torch.empty(B * n * S, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0x1234 + rank)
    view = buf.view(B, n, S)
    view[:, :k] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
    base = buf.data_ptr()
    table = (base + torch.arange(B * n, dtype=torch.int64, device=dev) * S).contiguous()
    lo, hi = shard_range(B * world, rank, world)  # this rank's global stripe indices
    fail = torch.from_numpy(failure_pairs(B, k, 0x1234 ^ lo).reshape(-1)).to(dev)
    batch = ec.make_batch(k, m, S, B, table)

    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step():
        ec.encode(batch, sh)
        ec.reconstruct(batch, fail, sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        ec.encode(batch, sh)
        ev[i][1].record(stream)
        ec.reconstruct(batch, fail, sh)
        ev[i][2].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()

    elapsed = t1 - t0
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    rec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    units = 2.0 * k * S * B * args.steps  # user-data bytes through both passes
    elapsed, units = reduce_timing(elapsed, units, dev)

    verified = None
    if not args.no_verify:
        # erase the two failed data strips of every stripe, reconstruct, compare
        good = view[:, :k].clone()
        f2 = fail.view(B, 2).long()
        si = torch.arange(B, device=dev)
        view[si, f2[:, 0]] = 0
        view[si, f2[:, 1]] = 0
        ec.reconstruct(batch, fail, sh)
        torch.cuda.synchronize(dev)
        verified = bool(torch.equal(view[:, :k], good))
        del good

    value = units / elapsed / GIB
    workload = f"raid6_{k}p{m}_{S // 1024}k"
    enc_bytes = float(n * S * B)          # algorithmic: k reads + 2 writes per stripe
    rec_bytes = float(n * S * B)          # k-2 data + P + Q reads, 2 writes per stripe
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    traffic, traffic_src = load_pmc_traffic(workload)

    out = {
        "metric": "GiB/s device-resident RAID6 8+2 encode+reconstruct, 64KiB strips, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch Generator seed 0x1234+rank)",
        "config": {
            "workload": f"RAID6 {k}+{m} P+Q encode + dual-data-failure reconstruct, "
                        f"{S // 1024} KiB strips, {B} stripes per GPU (configs[2])",
            "k": k, "m": m, "strip_bytes": S, "stripes_per_gpu": B,
            "layout": "stripe-major contiguous, device pointer table",
            "parallelism": f"stripe-sharded x{world}, no collectives",
        },
        "breakdown": {
            "encode_ms": round(enc_ms, 4),
            "reconstruct_ms": round(rec_ms, 4),
            "encode_user_gib_s": round(k * S * B / (enc_ms * 1e-3) / GIB, 1),
            "reconstruct_user_gib_s": round(k * S * B / (rec_ms * 1e-3) / GIB, 1),
            "encode_hbm_gb_s": round(enc_gbs, 1),
            "reconstruct_hbm_gb_s": round(rec_bytes / (rec_ms * 1e-3) / 1e9, 1),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": f"k_encode<K={k},M=2> (draid_ec_encode)",
            "achieved": round(enc_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": enc_bytes,
        },
        "verified_roundtrip": verified,
    }
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            try:
                threads = min(16, len(os.sched_getaffinity(0)))
            except AttributeError:
                threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(k, m, S, args.cpu_seconds, threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

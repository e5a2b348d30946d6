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
    """Contiguous stripe range [lo, hi) of a rank: stripes are independent, so ranks shard them
    with no collective on the data path."""
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


def failure_single(nstripes: int, k: int, seed: int) -> np.ndarray:
    """[nstripes, 2] one lost data index per stripe (x = splitmix-style draw mod k)."""
    rng = np.random.default_rng(seed)
    x = rng.integers(0, k, nstripes)
    return np.stack([x, np.full(nstripes, 0xFF)], axis=1).astype(np.uint8)


# BASELINE.json configs the harness can run.  The default (no --config) is the
# headline metric's workload; the others are measured with the same harness and
# reported beside it (they are not the driver's bench line).
CONFIGS = {
    # configs[2] -- the metric's workload: RAID6 8+2 encode + reconstruct at 64 KiB
    "raid6_8p2_64k": dict(k=8, m=2, strip_kib=64, stripes=4096, failures="dual",
                          label="RAID6 8+2 P+Q encode + dual-data-failure reconstruct, 64 KiB "
                                "strips (configs[2])"),
    # configs[1] -- RAID5 4+1 XOR encode (+ single-failure reconstruct), 64 KiB
    "raid5_4p1_64k": dict(k=4, m=1, strip_kib=64, stripes=4096, failures="single",
                          label="RAID5 4+1 XOR encode + single-failure reconstruct, 64 KiB "
                                "strips (configs[1])"),
    # configs[3] -- RAID6 8+2 single-failure degraded read, 128 KiB; strong scaling
    # (--strong) splits 16384 stripes (20 GiB) over the ranks
    "raid6_8p2_128k_single": dict(k=8, m=2, strip_kib=128, stripes=4096, strong_stripes=16384,
                                  failures="single",
                                  label="RAID6 8+2 encode + single-failure reconstruct, 128 KiB "
                                        "strips (configs[3])"),
    # configs[4] -- RAID6 16+2 dual failure, 256 KiB; 4096 stripes over 8 GPUs = 512 per GPU
    "raid6_16p2_256k_dual": dict(k=16, m=2, strip_kib=256, stripes=512, strong_stripes=4096,
                                 failures="dual",
                                 label="RAID6 16+2 encode + dual-data-failure reconstruct, 256 KiB "
                                       "strips (configs[4])"),
}


def reconstruct_bytes_per_stripe(k: int, m: int, S: int, failures: str) -> int:
    """Algorithmic HBM bytes of one stripe's reconstruct: every surviving strip it needs is
    read once, every lost strip written once."""
    if failures == "dual":
        return (k + 2) * S          # k-2 data + P + Q read, 2 written
    return (k + 1) * S              # k-1 data + P read, 1 written


def load_pmc(workload: str):
    """Per-launch HBM bytes of each kernel from the committed rocprofv3 PMC
    summary (profiles/pmc_<workload>.json, tools/collect_pmc.py), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        return json.load(f), os.path.relpath(path, ROOT)


def cpu_baseline(k: int, m: int, S: int, failures: str, seconds: float, threads: int) -> dict:
    """The CPU restatement of isa-l (oracle/) timed on the host cores on a bounded
    sample of the same workload: 64 stripes, encode + reconstruct.  Uses the
    AVX-512 (+GFNI affine) restatement of isa-l's x86 kernels when the host has
    them (oracle/isal_simd.c), else the scalar one; also times one core."""
    import oracle
    simd = oracle.simd_available()

    def sample(nstripes):
        buf = np.frombuffer(np.random.default_rng(1).bytes((k + m) * S * nstripes), np.uint8).copy()
        fail = (failure_pairs if failures == "dual" else failure_single)(nstripes, k, 7)
        return buf, fail.reshape(-1)

    def run(buf, fail, nstripes, nthr, secs):
        el, passes = oracle.bench_encode_reconstruct(buf, k, m, S, nstripes, S, (k + m) * S, fail,
                                                     True, nthr, secs, simd=simd)
        return (2.0 * k * S * nstripes * passes / el / GIB, passes, el) if el > 0 else (None, 0, el)

    B = 64  # cache-resident (tens of MiB): the CPU's best case
    buf, fail = sample(B)
    value, passes, el = run(buf, fail, B, threads, seconds)
    if value is None:
        return {"value": None, "error": "oracle bench failed"}
    one, _, _ = run(buf, fail, B, 1, max(1.0, seconds / 4))
    # every core the process may run on (the GPU box's share is 16 of them; the
    # host has many more, shared with other tenants), beside the 16 and the 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or threads
    allc = None
    if affinity > threads:
        allc, _, _ = run(buf, fail, B, min(affinity, 512), max(1.0, seconds / 4))
    # the same work streaming from DRAM, as the full-size workload would run on the host
    B2 = max(64, (1 << 30) // ((k + m) * S))
    del buf
    buf2, fail2 = sample(B2)
    dram, passes2, el2 = run(buf2, fail2, B2, threads, max(1.0, seconds / 2))
    del buf2
    impl = ("AVX-512BW + GFNI restatement of isa-l's pq_gen_avx512 / gf_vect_mul (affine "
            "constant multiply)" if simd else
            "64-bit SWAR restatement of isa-l pq_gen_base + nibble-table gf_vect_mul, -O3 -mavx2")
    return {"value": round(value, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "single_core_value": round(one, 3) if one else None,
            # every core this process may run on; when that is no more than `cores`
            # (the GPU box gives a one-GPU job 16) the two runs are the same run
            "all_cores_value": round(allc, 3) if allc else round(value, 3),
            "all_cores": min(affinity, 512) if allc else threads,
            "affinity_cores": affinity,
            "dram_resident_value": round(dram, 3) if dram else None,
            "dram_resident_sample": f"{B2} stripes ({(k + m) * S * B2 >> 20} MiB), {passes2} "
                                    f"passes in {el2:.1f}s, {threads} pthreads",
            "sample": f"{B} stripes x {k}+{m} x {S // 1024} KiB, encode + {failures}-failure "
                      f"reconstruct, {passes} passes in {el:.1f}s, C oracle ({impl}), "
                      f"{threads} pthreads"}


def run_single_process(args, torch, ec) -> None:
    """The same step with every device slot driven from one thread (draid_ec_mgpu):
    slot d holds B stripes in its GPU's HBM (weak scaling) -- the stripes a raid
    bdev would route to it by index -- and each step fans encode + reconstruct out
    over the slots' streams; no collective, no peer traffic."""
    cfg = CONFIGS[args.config]
    k, m, S = cfg["k"], cfg["m"], cfg["strip_kib"] * 1024
    n = k + m
    G = max(1, args.gpus)
    B = args.stripes or cfg["stripes"]
    ndev = torch.cuda.device_count()
    devices = [d % ndev for d in range(G)]
    ec.lib()
    mg = ec.MultiGpu(devices)
    fgen = failure_pairs if cfg["failures"] == "dual" else failure_single
    bufs, views, tables, batches, fails, fail_nps = [], [], [], [], [], []
    for d in range(G):
        dev = torch.device("cuda", devices[d])
        buf = torch.empty(B * n * S, dtype=torch.uint8, device=dev)
        g = torch.Generator(device=dev)
        g.manual_seed(0x1234 + d)
        view = buf.view(B, n, S)
        view[:, :k] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
        table = (buf.data_ptr() + torch.arange(B * n, dtype=torch.int64, device=dev) * S).contiguous()
        fnp = fgen(B, k, 0x1234 ^ (d * B))
        bufs.append(buf)
        views.append(view)
        tables.append(table)
        batches.append(ec.make_batch(k, m, S, B, table))
        fail_nps.append(fnp)
        fails.append(torch.from_numpy(fnp.reshape(-1)).to(dev))
    for d in range(ndev):
        torch.cuda.synchronize(d)

    def step():
        mg.encode(batches)
        mg.reconstruct(batches, fails)

    for _ in range(args.warmup):
        step()
    mg.synchronize()
    # per-kernel events on slot 0's stream (the stream its kernels are launched on)
    s0 = torch.cuda.ExternalStream(mg.stream(0), device=torch.device("cuda", devices[0]))
    # Two event records per step (before the encode, between the kernels); the record in
    # front of step i+1 also ends step i's reconstruct -- a record between two kernels costs
    # the stream a few microseconds, so none is made twice.
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    ev_end = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        # slot 0's kernels are bracketed by events; the other slots run the same step
        ev[i][0].record(s0)
        mg.encode(batches)
        ev[i][1].record(s0)
        mg.reconstruct(batches, fails)
    ev_end.record(s0)
    mg.synchronize()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    rec_ms = float(np.mean([ev[i][1].elapsed_time(ev[i + 1][0] if i + 1 < args.steps else ev_end)
                            for i in range(args.steps)]))
    verified = None
    if not args.no_verify:
        # erase the failed data strips of every stripe on every slot, rebuild, compare
        goods = []
        for d in range(G):
            dev = torch.device("cuda", devices[d])
            goods.append(views[d][:, :k].clone())
            si = torch.arange(B, device=dev)
            for slot in range(2):
                idx = np.nonzero(fail_nps[d][:, slot] != 0xFF)[0]
                if len(idx):
                    ii = torch.from_numpy(idx).to(dev)
                    lost = torch.from_numpy(fail_nps[d][idx, slot].astype(np.int64)).to(dev)
                    views[d][si[ii], lost] = 0
            torch.cuda.synchronize(dev)
        mg.reconstruct(batches, fails)
        mg.synchronize()
        verified = all(bool(torch.equal(views[d][:, :k], goods[d])) for d in range(G))
        del goods
    units = 2.0 * k * S * B * G * args.steps
    value = units / elapsed / GIB
    enc_bytes = float(n * S * B)
    rec_bytes = float(reconstruct_bytes_per_stripe(k, m, S, cfg["failures"]) * B)
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    rec_gbs = rec_bytes / (rec_ms * 1e-3) / 1e9
    pmc, pmc_src = load_pmc(args.config)
    dominant = "reconstruct" if rec_ms >= enc_ms else "encode"
    gbs = rec_gbs if dominant == "reconstruct" else enc_gbs
    out = {
        "metric": ("GiB/s device-resident RAID6 8+2 encode+reconstruct, 64KiB strips, 1/2/4/8 GPU"
                   if args.config == "raid6_8p2_64k" else f"GiB/s device-resident {cfg['label']}"),
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": G, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch Generator seed 0x1234+slot)",
        "config": {"workload": f"{cfg['label']}, {B} stripes per device slot", "name": args.config,
                   "k": k, "m": m, "strip_bytes": S, "stripes_per_gpu": B, "stripes_total": B * G,
                   "failures": cfg["failures"],
                   "layout": "stripe-major contiguous, device pointer table",
                   "parallelism": f"ONE process, {G} device slots on GPUs {devices} "
                                  "(draid_ec_mgpu), stripe-sharded, no collectives"},
        "breakdown": {"encode_ms_slot0": round(enc_ms, 4), "reconstruct_ms_slot0": round(rec_ms, 4),
                      "note": "slot 0's events include the host's launches on the other slots"},
        "roofline": {"bound": "hbm", "kernel": f"k_{dominant}<K={k},M={m}> on slot 0",
                     "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(gbs / HBM_PEAK_GBS, 4),
                     "traffic": (pmc or {}).get(f"{dominant}_hbm_bytes_per_launch"),
                     "traffic_source": pmc_src},
        "verified_roundtrip": verified, "cpu_baseline": None,
    }
    mg.close()
    print(json.dumps(out), flush=True)


COMPILED_K = tuple(range(2, 21))  # widths with unrolled kernels


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="raid6_8p2_64k", choices=sorted(CONFIGS))
    ap.add_argument("--shape", default=None, metavar="K,M,STRIP_KIB,STRIPES,FAILURES",
                    help="lab runs only: any stripe shape instead of a BASELINE config, "
                         "e.g. 6,2,64,4096,dual (never the driver's bench line)")
    ap.add_argument("--stripes", type=int, default=None,
                    help="stripes per GPU (override); with --strong, the whole job's")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: a fixed stripe count (the config's strong_stripes) "
                         "sharded across the ranks instead of a fixed count per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--dispatch-events", action="store_true",
                    help="time the kernels with events carried by each launch's own dispatch "
                         "instead of events recorded on the stream around them")
    ap.add_argument("--layout", default="stripe_major", choices=["stripe_major", "strip_major"],
                    help="placement of the stripes in HBM: stripe-major (one stripe-cache slot per "
                         "stripe) or strip-major (one region per strip index)")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--stripe-pad", type=int, default=0,
                    help="lab runs only: bytes added to the stripe pitch of the stripe-major layout "
                         "(stripe s at s * ((k+m) * S + pad)); 0 = the BASELINE layout")
    ap.add_argument("--strip-pad", type=int, default=0,
                    help="lab runs only: bytes added between the strips of a stripe")
    ap.add_argument("--single-process", action="store_true",
                    help="drive --gpus device slots from THIS process through draid_ec_mgpu (the "
                         "shape of an SPDK target: one process, stripes routed to GPUs by index) "
                         "instead of one rank per GPU; slots beyond the visible GPUs share them")
    ap.add_argument("--dist-backend", default="nccl",
                    help="backend of the timing collectives (nccl = RCCL; gloo only for "
                         "rehearsing several ranks on one GPU)")
    args = ap.parse_args()
    if args.variant:  # A/B kernel variants exist only in the lab build (tools/sweep.py)
        os.environ.setdefault("DRAID_EC_LIB",
                              os.path.join(ROOT, "draid-spdk_amd", "liblab", "libdraid_ec.so"))

    import torch
    import torch.distributed as dist
    import draid_ec as ec

    if args.single_process:
        run_single_process(args, torch, ec)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # One rank per GPU; with fewer visible GPUs than ranks (a rehearsal on a
    # single-GPU box) ranks share devices round-robin.
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ec.lib()
    ec.set_variant(args.variant)

    cfg = CONFIGS[args.config]
    if args.shape:
        sk, sm, skib, sb, sf = args.shape.split(",")
        if sf not in ("single", "dual") or (sf == "dual" and int(sm) != 2):
            ap.error("--shape: FAILURES is 'single' or 'dual' (dual needs M = 2)")
        args.config = f"shape_{sk}p{sm}_{skib}k_{sf}"
        cfg = dict(k=int(sk), m=int(sm), strip_kib=int(skib), stripes=int(sb), failures=sf,
                   label=f"lab shape {sk}+{sm} x {skib} KiB, {sf} failure")
    k, m, S = cfg["k"], cfg["m"], cfg["strip_kib"] * 1024
    if args.strong:  # fixed total, contiguous stripe ranges per rank
        total = args.stripes or cfg.get("strong_stripes", cfg["stripes"])
    else:            # weak scaling: B stripes per GPU
        total = (args.stripes or cfg["stripes"]) * world
    lo, hi = shard_range(total, rank, world)  # this rank's global stripe indices
    B = hi - lo
    n = k + m
    # Stripes in HBM.  stripe_major: stripe s = [D0 .. D{k-1} P Q], strips contiguous
    # (one stripe-cache slot per stripe); strip_major: one region per strip index j
    # holding strip j of every stripe.  The kernels only see the pointer table.
    strip_pitch = S + args.strip_pad
    stripe_pitch = n * strip_pitch + args.stripe_pad
    buf = torch.empty(B * stripe_pitch, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0x1234 + rank)
    base = buf.data_ptr()
    if args.layout == "stripe_major":
        # [stripe, strip, byte] over the (possibly padded) pitches
        view = buf.as_strided((B, n, S), (stripe_pitch, strip_pitch, 1))
        si = torch.arange(B, dtype=torch.int64, device=dev).repeat_interleave(n)
        sj = torch.arange(n, dtype=torch.int64, device=dev).repeat(B)
        table = (base + si * stripe_pitch + sj * strip_pitch).contiguous()
    else:
        view = buf.view(n, B, S).permute(1, 0, 2)  # [stripe, strip, byte] over the regions
        si = torch.arange(B, dtype=torch.int64, device=dev).repeat_interleave(n)
        sj = torch.arange(n, dtype=torch.int64, device=dev).repeat(B)
        table = (base + (sj * B + si) * S).contiguous()
    view[:, :k] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
    fgen = failure_pairs if cfg["failures"] == "dual" else failure_single
    fail_np = fgen(B, k, 0x1234 ^ lo)
    fail = torch.from_numpy(fail_np.reshape(-1)).to(dev)
    batch = ec.make_batch(k, m, S, B, table)

    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step():
        ec.encode(batch, sh)
        ec.reconstruct(batch, fail, sh)

    verified = None
    if not args.no_verify:
        # before anything is timed: encode, erase the failed data strips of every stripe,
        # reconstruct, compare
        ec.encode(batch, sh)
        torch.cuda.synchronize(dev)
        good = view[:, :k].clone()
        si = torch.arange(B, device=dev)
        for slot in range(2):
            idx = np.nonzero(fail_np[:, slot] != 0xFF)[0]
            if len(idx):
                ii = torch.from_numpy(idx).to(dev)
                view[si[ii], torch.from_numpy(fail_np[idx, slot].astype(np.int64)).to(dev)] = 0
        ec.reconstruct(batch, fail, sh)
        torch.cuda.synchronize(dev)
        verified = bool(torch.equal(view[:, :k], good))
        del good
        if world > 1:  # every rank's shard must come back
            vt = torch.tensor([1.0 if verified else 0.0], dtype=torch.float64,
                              device=dev if args.dist_backend == "nccl" else torch.device("cpu"))
            dist.all_reduce(vt, op=dist.ReduceOp.MIN)
            verified = bool(vt.item() == 1.0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # Per-kernel HIP events over the timed region: recorded on the stream around the
    # kernels, two per step (before the encode, between the kernels; the record in front of
    # step i+1 also ends step i's reconstruct -- a record between two kernels costs the
    # stream a few microseconds, 0.5% of this step, so none is made twice).
    # --dispatch-events: every launch carries its own start and stop event in its dispatch
    # instead (the runtime stamps them from the kernel's start and end): the durations are
    # then the kernels' alone, as a profiler reports them (8+2 x 64 KiB: 384.6 + 399.4 us
    # against 387.7 + 402.4 between records), but such a dispatch costs the stream more than
    # a record does and the step runs 0.6% longer (0.7953 vs 0.7902 ms), so it is not the
    # default.
    if args.dispatch_events:
        ev = [[ec.event_create() for _ in range(4)] for _ in range(args.steps)]
    else:
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
        ev_end = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if args.dispatch_events:
        for i in range(args.steps):
            ec.launch_events(ev[i][0], ev[i][1])
            ec.encode(batch, sh)
            ec.launch_events(ev[i][2], ev[i][3])
            ec.reconstruct(batch, fail, sh)
    else:
        for i in range(args.steps):
            ev[i][0].record(stream)
            ec.encode(batch, sh)
            ev[i][1].record(stream)
            ec.reconstruct(batch, fail, sh)
        ev_end.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()  # this rank's K steps; the job's time is the max over ranks below
    if world > 1:
        dist.barrier()

    elapsed = t1 - t0
    if args.dispatch_events:
        enc_all = [ec.event_elapsed_ms(e[0], e[1]) for e in ev]
        rec_all = [ec.event_elapsed_ms(e[2], e[3]) for e in ev]
        for e in ev:
            for x in e:
                ec.event_destroy(x)
    else:
        enc_all = [e[0].elapsed_time(e[1]) for e in ev]
        rec_all = [ev[i][1].elapsed_time(ev[i + 1][0] if i + 1 < args.steps else ev_end)
                   for i in range(args.steps)]
    enc_ms, rec_ms = float(np.mean(enc_all)), float(np.mean(rec_all))
    units = 2.0 * k * S * B * args.steps  # user-data bytes through both passes
    elapsed, units = reduce_timing(elapsed, units,
                                   dev if args.dist_backend == "nccl" else torch.device("cpu"))

    value = units / elapsed / GIB
    workload = args.config
    enc_bytes = float(n * S * B)  # algorithmic: k data read + m parity written per stripe
    rec_bytes = float(reconstruct_bytes_per_stripe(k, m, S, cfg["failures"]) * B)
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    rec_gbs = rec_bytes / (rec_ms * 1e-3) / 1e9
    pmc, pmc_src = load_pmc(workload)

    def roof(kind, gbs, nbytes):
        # the kernel the library launches for this width (csrc/ec_kernels.hip,
        # enc_split / rec_split): items shared by several waves from k = 3 (encode)
        # and k = 8 (reconstruct) up
        enc_k = "k_encode_split" if k >= 3 and k in COMPILED_K else "k_encode"
        rec_k = "k_reconstruct_cols" if k >= 8 and k in COMPILED_K else "k_reconstruct"
        name = (f"{enc_k}<K={k},M={m}> (draid_ec_encode)" if kind == "encode" else
                f"{rec_k}<K={k},M={m}> (draid_ec_reconstruct, {cfg['failures']} failure)")
        return {"bound": "hbm", "kernel": name, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                "traffic": (pmc or {}).get(f"{kind}_hbm_bytes_per_launch"),
                "traffic_source": pmc_src, "algorithmic_bytes_per_launch": nbytes}

    roofs = {"encode": roof("encode", enc_gbs, enc_bytes),
             "reconstruct": roof("reconstruct", rec_gbs, rec_bytes)}
    dominant = "reconstruct" if rec_ms >= enc_ms else "encode"
    metric = ("GiB/s device-resident RAID6 8+2 encode+reconstruct, 64KiB strips, 1/2/4/8 GPU"
              if workload == "raid6_8p2_64k" else f"GiB/s device-resident {cfg['label']}")

    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch Generator seed 0x1234+rank)",
        "config": {
            "workload": f"{cfg['label']}, " + (f"{total} stripes over {world} GPU(s)"
                                                 if args.strong else f"{B} stripes per GPU"),
            "name": workload, "k": k, "m": m, "strip_bytes": S, "stripes_per_gpu": B,
            "stripes_total": total,
            "failures": cfg["failures"],
            "layout": ("stripe-major contiguous" if args.layout == "stripe_major" else
                       "strip-major (one region per strip index)") + ", device pointer table" +
                      (f", stripe pitch +{args.stripe_pad} B, strip pitch +{args.strip_pad} B"
                       if args.stripe_pad or args.strip_pad else ""),
            "parallelism": f"stripe-sharded x{world}, no collectives",
        },
        **({"lab_variant": args.variant} if args.variant else {}),
        "breakdown": {
            "encode_ms": round(enc_ms, 4),
            "reconstruct_ms": round(rec_ms, 4),
            "encode_ms_median": round(float(np.median(enc_all)), 4),  # medians beside the means: a slow start does not hide
            "reconstruct_ms_median": round(float(np.median(rec_all)), 4),
            "encode_user_gib_s": round(k * S * B / (enc_ms * 1e-3) / GIB, 1),
            "reconstruct_user_gib_s": round(k * S * B / (rec_ms * 1e-3) / GIB, 1),
            "encode_hbm_gb_s": round(enc_gbs, 1),
            "reconstruct_hbm_gb_s": round(rec_gbs, 1),
        },
        "roofline": roofs[dominant],
        "roofline_other": roofs["encode" if dominant == "reconstruct" else "reconstruct"],
        "verified_roundtrip": verified,
    }
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            try:
                threads = min(16, len(os.sched_getaffinity(0)))
            except AttributeError:
                threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(k, m, S, cfg["failures"], args.cpu_seconds,
                                               threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

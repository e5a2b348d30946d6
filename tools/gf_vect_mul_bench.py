"""Throughput of the synchronous draid_gf_vect_mul (gf_vect_mul.c:108 call shape) on
device-resident buffers: per-call wall time (launch + kernel + stream wait) over sizes.
Prints one JSON line per size."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402

tbl = ec.gf_vect_mul_init(0x53)
for mib in (1, 16, 256, 1024):
    n = mib << 20
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda:0")
    dst = torch.empty_like(src)
    torch.cuda.synchronize()
    for _ in range(3):
        assert ec.gf_vect_mul(n, tbl, src, dst) == 0
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        ec.gf_vect_mul(n, tbl, src, dst)
    dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"op": "gf_vect_mul", "mib": mib, "us_per_call": round(dt * 1e6, 1),
                      "hbm_gb_s": round(2 * n / dt / 1e9, 1)}), flush=True)

#!/usr/bin/env python3
"""Host time one thread spends per batched launch (draid_ec_encode /
draid_ec_reconstruct at the headline shape, ctypes overhead included): the number
that decides how many GPUs one thread can keep busy.  Launches are issued in
bursts of 16 (8 GPUs x encode + reconstruct) behind a synchronize, so the queue is
never deep enough to block the host."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402

dev = torch.device("cuda", 0)
k, m, L, B = 8, 2, 65536, 4096
n = k + m
buf = torch.randint(0, 256, (B, n, L), dtype=torch.uint8, device=dev)
base = buf.data_ptr()
table = (torch.arange(B * n, dtype=torch.int64, device=dev) * L + base)
fail = torch.tensor([[1, 5]] * B, dtype=torch.uint8, device=dev)
batch = ec.make_batch(k, m, L, B, table)
s = ec.stream_create()
ec.encode(batch, s)
ec.stream_synchronize(s)
enc, rec, burst = [], [], []
for it in range(40):
    t_b = time.perf_counter()
    for g in range(8):
        t0 = time.perf_counter()
        ec.encode(batch, s)
        t1 = time.perf_counter()
        ec.reconstruct(batch, fail.data_ptr(), s)
        t2 = time.perf_counter()
        enc.append(t1 - t0)
        rec.append(t2 - t1)
    burst.append(time.perf_counter() - t_b)
    ec.stream_synchronize(s)
ec.stream_destroy(s)
us = lambda v, q: round(float(np.percentile(v[16:], q)) * 1e6, 2)
out = {"shape": "RAID6 8+2 x 64 KiB x 4096", "encode_call_us_p50": us(enc, 50), "encode_call_us_p99": us(enc, 99),
       "reconstruct_call_us_p50": us(rec, 50), "reconstruct_call_us_p99": us(rec, 99),
       "burst_of_16_launches_us_p50": round(float(np.median(burst[2:])) * 1e6, 1),
       "budget_us_per_launch_for_8_gpus": 49}
print(json.dumps(out))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "launch_rate.json"), "w"), indent=1)

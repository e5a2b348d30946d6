#!/usr/bin/env python3
"""Per-call latency of the synchronous isa-l-shaped calls and of one-stripe
batched launches (the low-queue-depth case an SPDK reactor sees)."""
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
res = []
for k, L in [(4, 65536), (8, 65536), (8, 4096), (16, 262144)]:
    n = k + 2
    b = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev)
    ptrs = [b[j].data_ptr() for j in range(n)]
    ec.pq_gen(ptrs, L)
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        ec.pq_gen(ptrs, L)
        ts.append(time.perf_counter() - t0)
    xs = []
    for _ in range(200):
        t0 = time.perf_counter()
        ec.xor_gen(ptrs[:k + 1], L)
        xs.append(time.perf_counter() - t0)
    cs = []
    for _ in range(200):
        t0 = time.perf_counter()
        assert ec.pq_check(ptrs, L) == 0
        cs.append(time.perf_counter() - t0)
    r = {"k": k, "len": L, "pq_gen_us_p50": round(np.median(ts) * 1e6, 1),
         "pq_check_us_p50": round(np.median(cs) * 1e6, 1),
         "pq_gen_us_p99": round(np.percentile(ts, 99) * 1e6, 1),
         "xor_gen_us_p50": round(np.median(xs) * 1e6, 1)}
    res.append(r)
    print(json.dumps(r), flush=True)
# one-stripe batched launch on a stream, polled like an SPDK poller
k, L = 8, 65536
n = k + 2
b = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev)
table = torch.tensor([b[j].data_ptr() for j in range(n)], dtype=torch.int64, device=dev)
batch = ec.make_batch(k, 2, L, 1, table)
s = ec.stream_create()
ts = []
for i in range(300):
    t0 = time.perf_counter()
    ec.encode(batch, s)
    while ec.stream_query(s) != 0:
        pass
    ts.append(time.perf_counter() - t0)
ec.stream_destroy(s)
r = {"batched_one_stripe_8p2_64k_poll_us_p50": round(np.median(ts[20:]) * 1e6, 1),
     "p99": round(np.percentile(ts[20:], 99) * 1e6, 1)}
res.append(r)
print(json.dumps(r), flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "latency.json"), "w"), indent=1)

#!/usr/bin/env python3
"""Where P and Q sit inside a stripe-major stripe: after the data (D0..Dk-1 P Q),
before it (P Q D0..Dk-1), or split (P D0..Dk-1 Q) -- encode and reconstruct
(random per-stripe failure pairs, as bench.py) through the pointer table."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
sys.path.insert(0, ROOT)
import draid_ec as ec  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
sh = st.cuda_stream


def timeit(fn, iters=10, rounds=7):
    ts = []
    for _ in range(rounds):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000 / iters)
    return float(np.median(ts))


out = []
for k, m, skib, B, failures in [(8, 2, 64, 4096, "dual"), (4, 1, 64, 4096, "single"),
                                (8, 2, 128, 4096, "single"), (16, 2, 256, 512, "dual")]:
    S = skib * 1024
    n = k + m
    buf = torch.empty(B * n * S, dtype=torch.uint8, device=dev).random_(0, 256)
    fgen = bench.failure_pairs if failures == "dual" else bench.failure_single
    fail = torch.from_numpy(fgen(B, k, 0x1234).reshape(-1)).to(dev)
    orders = {"data_then_parity": list(range(n)),
              "parity_first": list(range(m, n)) + list(range(m)),
              "P_data_Q": ([1 + j for j in range(k)] + [0] + ([n - 1] if m == 2 else []))}
    for name, pos in orders.items():
        # pos[j] = physical slot of logical strip j (j < k data, k = P, k+1 = Q)
        slots = torch.tensor(pos, dtype=torch.int64, device=dev)
        table = (buf.data_ptr() + (torch.arange(B, device=dev)[:, None] * n + slots[None, :]) * S)
        table = table.reshape(-1).contiguous()
        batch = ec.make_batch(k, m, S, B, table)
        enc = timeit(lambda: ec.encode(batch, sh))
        rec = timeit(lambda: ec.reconstruct(batch, fail, sh))
        rb = bench.reconstruct_bytes_per_stripe(k, m, S, failures) * B
        r = {"k": k, "m": m, "strip_kib": skib, "order": name,
             "enc_gb_s": round(n * S * B / enc / 1e3, 1), "rec_gb_s": round(rb / rec / 1e3, 1)}
        out.append(r)
        print(json.dumps(r), flush=True)
    del buf
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "layout_order.json"), "w"), indent=1)

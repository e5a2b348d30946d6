#!/usr/bin/env python3
"""Same stripes, same kernel body, three address sources: the device pointer
table (draid_ec_encode), the strided descriptor (draid_ec_encode_strided), and
the no-arithmetic stripe-pattern probe -- isolates what the pointer table and
the GF work cost at each strip size."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402

P = C.CDLL(os.path.join(ROOT, "tools", "probe", "libprobe.so"))
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
sh = st.cuda_stream
sink = torch.empty(1 << 20, dtype=torch.uint8, device=dev)


def timeit(fn, iters=10, rounds=5):
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
for k, m, skib, B in [(8, 2, 64, 4096), (8, 2, 128, 2048), (8, 2, 128, 4096), (16, 2, 256, 512),
                      (4, 1, 64, 4096)]:
    S = skib * 1024
    n = k + m
    buf = torch.empty(B * n * S, dtype=torch.uint8, device=dev).random_(0, 256)
    table = buf.data_ptr() + torch.arange(B * n, dtype=torch.int64, device=dev) * S
    batch = ec.make_batch(k, m, S, B, table)
    fail = torch.from_numpy(np.array([[0, 1]] * B if m == 2 else [[0, 255]] * B,
                                     np.uint8).reshape(-1)).to(dev)
    nbytes = n * S * B
    rbytes = (k + 2 if m == 2 else k + 1) * S * B
    r = {"k": k, "m": m, "strip_kib": skib, "stripes": B}
    r["enc_table"] = nbytes / timeit(lambda: ec.encode(batch, sh)) / 1e3
    r["enc_strided"] = nbytes / timeit(
        lambda: ec.encode_strided(buf, k, m, S, B, S, n * S, sh)) / 1e3
    r["rec_table"] = rbytes / timeit(lambda: ec.reconstruct(batch, fail, sh)) / 1e3
    r["rec_strided"] = rbytes / timeit(
        lambda: ec.reconstruct_strided(buf, k, m, S, B, S, n * S, fail, sh)) / 1e3
    r["probe"] = nbytes / timeit(lambda: P.probe_stripe_pattern(
        C.c_void_p(buf.data_ptr()), C.c_uint64(S), C.c_uint64(S), C.c_uint64(n * S), k, m, B,
        C.c_void_p(sink.data_ptr()), C.c_void_p(sh))) / 1e3
    r = {a: (round(b, 1) if isinstance(b, float) else b) for a, b in r.items()}
    out.append(r)
    print(json.dumps(r), flush=True)
    del buf, table
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "table_vs_strided.json"), "w"), indent=1)

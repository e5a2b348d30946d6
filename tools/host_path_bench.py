#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-resident stripe path.

Stripes live in pinned host memory (what SPDK's registered hugepage buffers
are); by default draid_ec_host_encode / _reconstruct read the strips
in place over PCIe (one launch over the mapped host range); with
DRAID_EC_HOST_STAGED they copy the strips into HBM chunk by chunk (encode: k in,
m out; reconstruct: k+m in, the rebuilt strips out).  Reported next to -- never instead of -- the
device-resident bench value.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import draid_ec as ec
    import bench
    k, m, S, B = 8, 2, 65536, int(os.environ.get("HOST_STRIPES", "4096"))
    n = k + m
    torch.cuda.init()
    t = torch.empty(B * n * S, dtype=torch.uint8).pin_memory()
    t.view(B, n, S)[:, :k] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8)
    fail = bench.failure_pairs(B, k, 0x1234).reshape(-1).copy()
    res = []
    for chunk in (0, 16, 32, 64, 128, 256):
        flags = 0 if chunk == 0 else ec.HOST_STAGED   # 0: mapped, read in place
        for op in ("encode", "reconstruct"):
            fn = (lambda: ec.host_encode(t, k, m, S, B, S, n * S, chunk, flags)) \
                if op == "encode" else \
                (lambda: ec.host_reconstruct(t, k, m, S, B, S, n * S, fail.ctypes.data, chunk,
                                             flags))
            fn()
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            sec = float(np.median(ts))
            h2d = (k if op == "encode" or chunk == 0 else n) * S * B
            d2h = (m if op == "encode" else 2) * S * B
            r = {"op": op, "mode": "mapped" if chunk == 0 else "staged",
                 "chunk_stripes": chunk, "seconds": round(sec, 4),
                 "user_gib_s": round(k * S * B / sec / 2**30, 2),
                 "h2d_gb_s": round(h2d / sec / 1e9, 2), "d2h_gb_s": round(d2h / sec / 1e9, 2)}
            res.append(r)
            print(json.dumps(r), flush=True)
    # mapped and staged agree: re-encode staged and compare P/Q
    ref = t.view(B, n, S)[:, k:].clone()
    assert ec.host_encode(t, k, m, S, B, S, n * S, 64, ec.HOST_STAGED) == 0
    assert torch.equal(ref, t.view(B, n, S)[:, k:]), "mapped and staged encode differ"
    out = os.path.join(ROOT, "gpurun_out", "host_path.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"config": {"k": k, "m": m, "strip": S, "stripes": B,
                              "memory": "torch pin_memory (hipHostMalloc)"}, "results": res}, f,
                  indent=1)


if __name__ == "__main__":
    main()

"""How a launch on host memory depends on the workgroups it runs in: B RAID6 8+2 x 64 KiB
stripes in pinned host memory through a host-pointer context (encode_sg / reconstruct_sg,
flush, synchronize), microseconds per flush and wait.  Such launches run the work lists'
looping kernels; DRAID_EC_HOST_GRID sets their workgroups (default: one per CU; 0: one per
work item, so nothing loops).  One JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402

k, m, S = 8, 2, 65536
n = k + m
ec.lib()
torch.cuda.init()
out = {"grid": os.environ.get("DRAID_EC_HOST_GRID", "CUs")}
for B in (4, 16, 32, 64, 256, 1024):
    host = torch.empty(B * n * S, dtype=torch.uint8).pin_memory()
    host.view(B, n, S)[:, :k] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8)
    base = host.data_ptr()
    ctx = ec.Ctx()
    ctx.set_host_pointers(True)
    lists = [[[(base + (s * n + j) * S, S)] for j in range(n)] for s in range(B)]
    for op in ("enc", "rec"):
        ts = []
        for rep in range(60 if B <= 64 else 12):
            for s in range(B):
                if op == "enc":
                    ctx.encode_sg(k, m, lists[s], S)
                else:
                    ctx.reconstruct_sg(k, m, lists[s], S, [s % k, (s + 3) % k])
            t0 = time.perf_counter()
            ctx.flush()
            ctx.synchronize()
            ts.append(time.perf_counter() - t0)
        out[f"{op}{B}"] = round(float(np.median(ts[len(ts) // 6:])) * 1e6, 1)
    ctx.close()
print(json.dumps(out), flush=True)

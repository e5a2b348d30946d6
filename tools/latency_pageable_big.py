import sys, time, json, os
import numpy as np
sys.path.insert(0, "draid-spdk_amd")
import torch
import draid_ec as ec
ec.lib(); torch.cuda.init()
for n, L in ((10, 1 << 20), (10, 4 << 20), (3, 16 << 20)):
    a = [np.random.randint(0, 256, L, dtype=np.uint8) for _ in range(n)]
    ptrs = [x.ctypes.data for x in a]
    f = (lambda: ec.xor_gen(ptrs, L)) if n == 3 else (lambda: ec.pq_gen(ptrs, L))
    f(); f()
    ts = []
    for _ in range(20):
        t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
    print(json.dumps({"bounce_max": os.environ.get("DRAID_EC_BOUNCE_MAX", "8MiB"), "vects": n, "len": L, "us": round(float(np.median(ts)) * 1e6, 1)}), flush=True)

import sys, time, json
import numpy as np
sys.path.insert(0, "draid-spdk_amd"); sys.path.insert(0, ".")
import torch
import draid_ec as ec
import bench
ec.lib(); torch.cuda.init()
k, m, S, B = 8, 2, 65536, 2048
n = k + m
a = np.random.randint(0, 256, B * n * S, dtype=np.uint8)
fail = bench.failure_pairs(B, k, 0x1234).reshape(-1).copy()
class W:  # minimal tensor-like for ec.host_encode
    pass
for chunk in (64, 128, 256):
    for op in ("encode", "reconstruct"):
        fn = (lambda: ec.host_encode(a.ctypes.data, k, m, S, B, S, n * S, chunk, 0)) if op == "encode" else \
             (lambda: ec.host_reconstruct(a.ctypes.data, k, m, S, B, S, n * S, fail.ctypes.data, chunk, 0))
        fn()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter(); fn(); ts.append(time.perf_counter() - t0)
        sec = float(np.median(ts))
        print(json.dumps({"memory": "pageable", "op": op, "chunk": chunk, "user_gib_s": round(k * S * B / sec / 2**30, 2)}), flush=True)

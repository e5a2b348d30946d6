import json, os, sys
import numpy as np
sys.path.insert(0, "draid-spdk_amd")
import torch
import draid_ec as ec
ec.lib()
k, m, S = 8, 2, 65536
n = k + m
dev = torch.device("cuda", 0)
B = 16
R = 32
host = torch.empty(R * B * n * S, dtype=torch.uint8).pin_memory()
host.view(R * B, n, S)[:, :k] = torch.randint(0, 256, (R * B, k, S), dtype=torch.uint8)
hbase = ec.device_pointer(host.data_ptr(), host.numel())
stream = torch.cuda.current_stream(dev); sh = stream.cuda_stream
batches = []
for r in range(R):
    tab = hbase + (np.arange(B * n, dtype=np.int64) + r * B * n) * S
    t = torch.from_numpy(tab).to(dev)
    batches.append((ec.make_batch(k, m, S, B, t), t))
for mode in ("same", "rotate", "same", "rotate"):
    ts = []
    for i in range(64):
        b = batches[0 if mode == "same" else i % R][0]
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream); ec.encode(b, sh); e.record(stream); torch.cuda.synchronize(dev)
        ts.append(a.elapsed_time(e) * 1e3)
    print(mode, "median us", round(float(np.median(ts[8:])), 1), "min", round(min(ts[8:]), 1))

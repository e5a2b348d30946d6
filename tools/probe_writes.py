#!/usr/bin/env python3
"""Write-only HBM rate by workgroup shape and store policy
(tools/probe/hbm_probe.hip:k_write_items), next to hipMemsetAsync."""
import ctypes as C
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = C.CDLL(os.path.join(ROOT, "tools", "probe", "libprobe.so"))
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
nbytes = 2560 << 20
buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
hip = C.CDLL("libamdhip64.so")


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


res = []
for nthr, vpl in [(64, 1), (64, 4), (256, 1), (256, 4), (1024, 1)]:
    for nt in (1, 0):
        us = timeit(lambda: L.probe_write_items(C.c_void_p(buf.data_ptr()), C.c_uint64(nbytes),
                                                nthr, vpl, nt, C.c_void_p(st.cuda_stream)))
        r = {"kernel": f"write_items {nthr}x{vpl} {'nt' if nt else 'plain'}",
             "gb_s": round(nbytes / us / 1e3, 1)}
        res.append(r)
        print(json.dumps(r), flush=True)
us = timeit(lambda: hip.hipMemsetAsync(C.c_void_p(buf.data_ptr()), 0x5a, C.c_size_t(nbytes),
                                       C.c_void_p(st.cuda_stream)))
res.append({"kernel": "hipMemsetAsync", "gb_s": round(nbytes / us / 1e3, 1)})
print(json.dumps(res[-1]), flush=True)
us = timeit(lambda: buf.fill_(7))
res.append({"kernel": "torch fill_", "gb_s": round(nbytes / us / 1e3, 1)})
print(json.dumps(res[-1]), flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "probe_writes.json"), "w"), indent=1)

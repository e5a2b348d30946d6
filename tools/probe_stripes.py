#!/usr/bin/env python3
"""Memory-pattern probe (tools/probe/hbm_probe.hip:k_stripe_pattern): HBM rate of
the encode access pattern without GF math, by strip size and layout padding."""
import ctypes as C
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = C.CDLL(os.path.join(ROOT, "tools", "probe", "libprobe.so"))
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
sink = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
res = []
CASES = os.environ.get("PROBE_CASES")
for (K, M, S_kib, B, gap_kib) in (json.loads(CASES) if CASES else [(8, 2, 64, 4096, 0), (8, 2, 128, 2048, 0), (8, 2, 128, 4096, 0),
                                  (8, 2, 256, 1024, 0), (16, 2, 64, 2048, 0), (16, 2, 256, 512, 0),
                                  (8, 2, 128, 4096, 4), (16, 2, 256, 512, 4), (8, 0, 64, 4096, 0),
                                  (8, 0, 128, 4096, 0), (16, 0, 256, 512, 0), (8, 2, 32, 8192, 0),
                                  (8, 2, 16, 16384, 0)]):
    S = S_kib * 1024
    stride = S + int(gap_kib * 1024)
    buf = torch.empty(B * (K + max(M, 2)) * stride + (1 << 20), dtype=torch.uint8, device=dev)
    buf.random_(0, 256)
    fn = lambda: L.probe_stripe_pattern(C.c_void_p(buf.data_ptr()), C.c_uint64(S),  # noqa
                                        C.c_uint64(stride),
                                        C.c_uint64((K + max(M, 2)) * stride), K, M, B,
                                        C.c_void_p(sink.data_ptr()), C.c_void_p(st.cuda_stream))
    ts = []
    for _ in range(5):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 100)  # us per launch
    us = float(np.median(ts))
    nbytes = (K + M) * S * B
    r = {"K": K, "M": M, "strip_kib": S_kib, "gap_kib": gap_kib, "stripes": B, "us": round(us, 1),
         "gb_s": round(nbytes / us / 1e3, 1)}
    res.append(r)
    print(json.dumps(r), flush=True)
    del buf
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "probe_stripes.json"), "w"), indent=1)

import json, os, sys, ctypes
import numpy as np
sys.path.insert(0, "draid-spdk_amd")
import torch
import draid_ec as ec
L = ec.lib()
L.draid_ec_test_launch_lds.argtypes = [ctypes.c_uint32]
L.draid_ec_test_launch_lds.restype = None
k, m, S = 8, 2, 65536
n = k + m
dev = torch.device("cuda", 0)
print("max LDS per block", torch.cuda.get_device_properties(0).shared_memory_per_block if hasattr(torch.cuda.get_device_properties(0), "shared_memory_per_block") else "?")
Bmax = 1024
host = torch.empty(Bmax * n * S, dtype=torch.uint8).pin_memory()
host.view(Bmax, n, S)[:, :k] = torch.randint(0, 256, (Bmax, k, S), dtype=torch.uint8)
hbase = ec.device_pointer(host.data_ptr(), host.numel())
devbuf = torch.randint(0, 256, (Bmax * n * S,), dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream(dev); sh = stream.cuda_stream
fail = torch.from_numpy(np.array([[s % k, (s + 3) % k] for s in range(Bmax)], np.uint8).reshape(-1)).to(dev)
for where, base in (("host", hbase), ("device", devbuf.data_ptr())):
    for B in (4, 16, 32, 64, 256, 1024):
        tab = base + np.arange(B * n, dtype=np.int64) * S
        t = torch.from_numpy(tab).to(dev)
        batch = ec.make_batch(k, m, S, B, t)
        row = {}
        for lds in (0, 16384, 32768, 49152, 57344, 65536 - 8192 - 2048, 98304, 131072):
            L.draid_ec_test_launch_lds(lds)
            try:
                for op in ("enc", "rec"):
                    ts = []
                    for i in range(24 if B <= 64 else 8):
                        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a.record(stream)
                        rc = ec.encode(batch, sh) if op == "enc" else ec.reconstruct(batch, fail, sh)
                        e.record(stream); torch.cuda.synchronize(dev)
                        ts.append(a.elapsed_time(e) * 1e3)
                    row[f"{op}@{lds//1024}K"] = round(float(np.median(ts[3:])), 1)
            except Exception as ex:
                row[f"@{lds//1024}K"] = "launch failed"
        L.draid_ec_test_launch_lds(0)
        print(json.dumps({"where": where, "stripes": B, **row}), flush=True)

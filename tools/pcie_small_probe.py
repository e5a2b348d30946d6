#!/usr/bin/env python3
"""How well does a SMALL launch drive the PCIe link?  RAID6 8+2 x 64 KiB stripes in
pinned host memory, B stripes per launch through the batched pointer-table call,
timed with events on the launch stream:
  parity "host"    P and Q written back over PCIe (what the raid module does)
  parity "device"  P and Q written to HBM (reads cross the link, writes do not)
The difference is what the write-back adds to a launch of that size."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))


def main():
    import torch
    import draid_ec as ec
    ec.lib()
    k, m, S = 8, 2, 65536
    n = k + m
    Bmax = 1024
    dev = torch.device("cuda", 0)
    host = torch.empty(Bmax * n * S, dtype=torch.uint8).pin_memory()
    host.view(Bmax, n, S)[:, :k] = torch.randint(0, 256, (Bmax, k, S), dtype=torch.uint8)
    hbase = ec.device_pointer(host.data_ptr(), host.numel())
    par = torch.zeros(Bmax * m * S, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    out = []
    for B in (1, 2, 4, 8, 16, 32, 64, 128, 256, 1024):
        for where in ("host", "device"):
            tab = np.empty((B, n), np.int64)
            for s in range(B):
                for j in range(n):
                    if j < k or where == "host":
                        tab[s, j] = hbase + (s * n + j) * S
                    else:
                        tab[s, j] = par.data_ptr() + (s * m + (j - k)) * S
            table = torch.from_numpy(tab.reshape(-1)).to(dev)
            batch = ec.make_batch(k, m, S, B, table)
            for _ in range(5):
                ec.encode(batch, sh)
            torch.cuda.synchronize(dev)
            reps = 40 if B <= 64 else 10
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(reps)]
            for a, b in ev:
                a.record(stream)
                ec.encode(batch, sh)
                b.record(stream)
                torch.cuda.synchronize(dev)
            us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
            r = {"stripes": B, "parity": where, "us": round(us, 1),
                 "us_per_stripe": round(us / B, 2),
                 "read_gb_s": round(k * S * B / us / 1e3, 1)}
            out.append(r)
            print(json.dumps(r), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pcie_small_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def two_streams():
    """Two launches of B stripes each: back to back on one stream, or side by side on
    two -- does running them together hide the fixed cost of a launch?"""
    import time
    import torch
    import draid_ec as ec
    ec.lib()
    k, m, S = 8, 2, 65536
    n = k + m
    dev = torch.device("cuda", 0)
    Bmax = 128
    host = torch.empty(2 * Bmax * n * S, dtype=torch.uint8).pin_memory()
    host.view(2 * Bmax, n, S)[:, :k] = torch.randint(0, 256, (2 * Bmax, k, S), dtype=torch.uint8)
    hbase = ec.device_pointer(host.data_ptr(), host.numel())
    s1, s2 = ec.stream_create(), ec.stream_create()
    for B in (8, 16, 32, 64):
        batches = []
        for half in range(2):
            tab = hbase + (np.arange(B * n, dtype=np.int64) + half * Bmax * n) * S
            table = torch.from_numpy(tab).to(dev)
            batches.append((ec.make_batch(k, m, S, B, table), table))
        torch.cuda.synchronize(dev)
        res = {}
        for mode in ("one_stream", "two_streams"):
            ts = []
            for r in range(45):
                t0 = time.perf_counter()
                ec.encode(batches[0][0], s1)
                ec.encode(batches[1][0], s1 if mode == "one_stream" else s2)
                ec.stream_synchronize(s1)
                ec.stream_synchronize(s2)
                ts.append(time.perf_counter() - t0)
            res[mode] = round(float(np.median(ts[5:])) * 1e6, 1)
        print(json.dumps({"stripes_per_launch": B, "launches": 2, **{f"{k_}_us": v for k_, v in res.items()}}),
              flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "two":
    two_streams()

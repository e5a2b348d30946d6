"""What separates the dual reconstruct from the encode at the headline shape (RAID6 8+2 x
64 KiB x 4096 stripes): the kernel, or where its reads and writes fall?  Times the encode
beside reconstructs with the same lost pair in every stripe -- (P, Q) moves exactly the
encode's bytes (all data in, P and Q out) through the reconstruct kernel; (0, 1) and (6, 7)
write two neighbouring data strips, (0, 4) two distant ones -- and beside a random data
pair per stripe (the bench's workload) and a single lost strip.  Rounds interleaved; one
JSON line with the medians."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402

k, m, S, B = 8, 2, 65536, 4096
dev = "cuda:0"
st = torch.cuda.current_stream().cuda_stream
pitch = (k + m) * S
buf = torch.randint(0, 256, (B * pitch,), dtype=torch.uint8, device=dev)
ptrs = (buf.data_ptr() + np.arange(B, dtype=np.int64)[:, None] * pitch +
        np.arange(k + m, dtype=np.int64)[None, :] * S)
table = torch.from_numpy(ptrs.reshape(-1)).to(dev)
batch = ec.make_batch(k, m, S, B, table)
rng = np.random.default_rng(3)
cases = {"encode": None}
for name, pair in (("pq", [k, k + 1]), ("0_1", [0, 1]), ("6_7", [6, 7]), ("0_4", [0, 4]),
                   ("3_q", [3, k + 1]), ("3_p", [3, k]), ("single_3", [3, 0xFF]), ("p_only", [k, 0xFF])):
    cases[name] = torch.from_numpy(np.tile(np.array(pair, np.uint8), (B, 1)).reshape(-1)).to(dev)
rand = np.stack([rng.permutation(k)[:2] for _ in range(B)]).astype(np.uint8)
cases["random_pair"] = torch.from_numpy(rand.reshape(-1)).to(dev)
rs = rng.integers(0, k, B).astype(np.uint8)
cases["random_single"] = torch.from_numpy(np.stack([rs, np.full(B, 0xFF, np.uint8)], 1).reshape(-1)).to(dev)


def run(f):
    if f is None:
        ec.encode(batch, st)
    else:
        ec.reconstruct(batch, f, st)


times = {n: [] for n in cases}
for _ in range(30):  # past the start-up clock dip
    run(None)
    run(cases["random_pair"])
torch.cuda.synchronize()
for rnd in range(7):
    for n, f in cases.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            run(f)
        a.record()
        for _ in range(20):
            run(f)
        b.record()
        torch.cuda.synchronize()
        times[n].append(a.elapsed_time(b) / 20 * 1e3)
print(json.dumps({"shape": "8+2 x 64 KiB x 4096", "median_us": {n: round(float(np.median(t)), 1) for n, t in times.items()}}))

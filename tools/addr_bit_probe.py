"""Which address bits must vary for HBM traffic to run at full rate?  A RAID5 2+1
encode over a crafted pointer table: per stripe two 16 KiB data strips are read and one
parity strip is written.  One side (the written strips, or the read strips) is confined
to addresses whose bit b is 0 -- every other block of 2^b bytes -- while the other side
streams over a contiguous region; b = none is the unconfined run.  One JSON line per
case (GB/s of read + write traffic)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402

S, B = 16384, 65536            # 1 GiB of parity, 2 GiB of data per launch
dev = "cuda:0"
st = torch.cuda.current_stream().cuda_stream
pool = torch.zeros(8 << 30, dtype=torch.uint8, device=dev)
base = (pool.data_ptr() + (1 << 30) - 1) & ~((1 << 30) - 1)   # 1 GiB aligned
assert base + (6 << 30) <= pool.data_ptr() + pool.numel()


def confined(n, b):
    """n strip addresses (offsets) of S bytes walking upwards through blocks with bit b = 0."""
    i = np.arange(n, dtype=np.int64) * S
    if b is None:
        return i
    blk = 1 << b
    return (i // blk) * (2 * blk) + (i % blk)


def run(side, b):
    spread0 = np.arange(B, dtype=np.int64) * (2 * S)
    if side == "write":
        d0, d1, p = spread0, spread0 + S, (4 << 30) // 2 + confined(B, b)   # parity from 2 GiB up
    else:
        c = confined(2 * B, b)
        d0, d1, p = c[0::2], c[1::2], (4 << 30) + np.arange(B, dtype=np.int64) * S
    tab = np.stack([base + d0, base + d1, base + p], axis=1).reshape(-1)
    assert tab.max() + S <= base + (6 << 30)
    table = torch.from_numpy(tab).to(dev)
    batch = ec.make_batch(2, 1, S, B, table)
    for _ in range(3):
        ec.encode(batch, st)
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        ec.encode(batch, st)
    e.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(e) / 10 * 1e3
    print(json.dumps({"confined": side, "bit": b, "us": round(us, 1),
                      "gb_s": round(3 * S * B / us / 1e3, 1)}), flush=True)


run("write", None)
for b in range(14, 28):
    run("write", b)
for b in range(14, 28):
    run("read", b)

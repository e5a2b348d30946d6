"""Is the slow encode of a power-of-two stripe pitch (6+2 x 64 KiB = 512 KiB) a WRITE
hot spot?  The encode writes P and Q at the same offset of every stripe; the
reconstruct writes wherever the lost strips are.  Times the reconstruct with the same
lost pair in every stripe against a random pair per stripe, beside the encode, for a
padded and an unpadded pitch.  One JSON line per case."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402

k, m, S, B = 6, 2, 65536, 5120
dev = "cuda:0"
st = torch.cuda.current_stream().cuda_stream


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for pad in (0, 16384):
    pitch = (k + m) * S + pad
    buf = torch.randint(0, 256, (B * pitch,), dtype=torch.uint8, device=dev)
    ptrs = (buf.data_ptr() + np.arange(B, dtype=np.int64)[:, None] * pitch +
            np.arange(k + m, dtype=np.int64)[None, :] * S)
    table = torch.from_numpy(ptrs.reshape(-1)).to(dev)
    batch = ec.make_batch(k, m, S, B, table)
    rng = np.random.default_rng(3)
    same = np.tile(np.array([1, 4], np.uint8), (B, 1))
    rand = np.stack([rng.permutation(k)[:2] for _ in range(B)]).astype(np.uint8)
    f_same = torch.from_numpy(same.reshape(-1)).to(dev)
    f_rand = torch.from_numpy(rand.reshape(-1)).to(dev)
    out = {"shape": "6+2 x 64 KiB x 5120", "stripe_pad": pad,
           "encode_us": round(timed(lambda: ec.encode(batch, st)), 1),
           "reconstruct_same_pair_us": round(timed(lambda: ec.reconstruct(batch, f_same, st)), 1),
           "reconstruct_random_pair_us": round(timed(lambda: ec.reconstruct(batch, f_rand, st)), 1)}
    print(json.dumps(out), flush=True)

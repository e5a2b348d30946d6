"""Why a power-of-two stripe pitch (6+2 x 64 KiB = 512 KiB) encodes slowly: a WRITE hot
spot on one address bit.  The encode writes P and Q at the same offset of every stripe;
a reconstruct with the same lost pair in every stripe writes two chosen strips of every
period.  Times such reconstructs for pairs inside one 256 KiB half of the period and
pairs that straddle it, beside the encode and a random pair per stripe, for an unpadded
and a padded pitch.  One JSON line per pitch."""
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
    extra = {}
    for name, pair in (("pq", [k, k + 1]), ("first_two", [0, 1]), ("last_two_data", [k - 2, k - 1]),
                       ("0_2", [0, 2]), ("0_4", [0, 4]), ("2_3", [2, 3]), ("1_3", [1, 3]),
                       ("3_4", [3, 4]), ("2_q", [2, k + 1])):
        f = torch.from_numpy(np.tile(np.array(pair, np.uint8), (B, 1)).reshape(-1)).to(dev)
        extra[f"reconstruct_{name}_us"] = round(timed(lambda f=f: ec.reconstruct(batch, f, st)), 1)
    out = {"shape": "6+2 x 64 KiB x 5120", "stripe_pad": pad, **extra,
           "encode_us": round(timed(lambda: ec.encode(batch, st)), 1),
           "reconstruct_same_pair_us": round(timed(lambda: ec.reconstruct(batch, f_same, st)), 1),
           "reconstruct_random_pair_us": round(timed(lambda: ec.reconstruct(batch, f_rand, st)), 1)}
    print(json.dumps(out), flush=True)

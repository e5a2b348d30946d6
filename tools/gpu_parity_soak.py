"""Randomised parity sweep on the GPU: many (k, m, strip length, batch, alignment)
combinations of the batched encode and reconstruct against the CPU oracle, beyond the
fixed grid of tests/test_gpu_parity.py.  Prints one line per 50 cases; exits non-zero
at the first mismatch, naming the case."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import draid_ec as ec  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import Batch, _random_failures, dev, host, oracle_encode  # noqa: E402

cases = int(sys.argv[1]) if len(sys.argv) > 1 else 400
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 20261113)
stream = torch.cuda.current_stream().cuda_stream
lens = [1, 7, 16, 48, 1000, 1024, 1040, 2048 + 16, 4096, 4096 + 5, 12 * 1024, 65536, 65536 + 3]
for c in range(cases):
    # four in five up to 32 (every unrolled width), the rest run-time widths up to 69
    k = int(rng.integers(2, 33)) if rng.random() < 0.8 else int(rng.integers(33, 70))
    m = int(rng.integers(1, 3))
    L = int(rng.choice(lens)) if rng.random() < 0.7 else int(rng.integers(1, 20000))
    B = int(rng.integers(1, 40))
    aligned = rng.random() < 0.7
    gap = int(16 + (-L) % 16) if aligned else int(rng.integers(0, 9))
    offset = 0 if aligned else int(rng.integers(0, 16))
    case = f"case {c}: k={k} m={m} L={L} B={B} gap={gap} offset={offset}"
    b = Batch(k, m, L, B, gap=gap, offset=offset, seed=c)
    before = host(b.strips())
    assert ec.encode(b.batch(ec), stream) == 0, case
    torch.cuda.synchronize()
    good = host(b.strips())
    if not (good == oracle_encode(before, k, m)).all():
        print("ENCODE MISMATCH", case, flush=True)
        sys.exit(1)
    fail = _random_failures(rng, B, k, m)
    v = b.strips()
    for s in range(B):
        for f in fail[s]:
            if f != 0xFF:
                v[s, int(f)].fill_(0x77)
    assert ec.reconstruct(b.batch(ec), dev(fail.reshape(-1)), stream) == 0, case
    torch.cuda.synchronize()
    if not (host(b.strips()) == good).all():
        print("RECONSTRUCT MISMATCH", case, flush=True)
        sys.exit(1)
    if gap and not (host(b.view()[:, :, L:]) == 0).all():
        print("GAP TOUCHED", case, flush=True)
        sys.exit(1)
    if (c + 1) % 50 == 0:
        print(f"{c + 1} cases ok (last: {case})", flush=True)
print(f"parity soak: {cases} random cases bit-exact against the oracle")

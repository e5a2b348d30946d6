"""Randomised sweep of the looping kernels: stripes in pinned HOST memory through a context
that resolves host pointers (encode, then reconstruct of random failure sets), random
widths, lengths, stripe counts, alignments and gaps, enough work items in most cases for the
kernels to loop (more items than CUs).  Against the CPU oracle; exits non-zero at the first
mismatch, naming the case."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "draid-spdk_amd"))
import draid_ec as ec  # noqa: E402
import oracle  # noqa: E402

cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 8128)
ec.lib()
torch.cuda.init()
for c in range(cases):
    k = int(rng.integers(2, 33)) if rng.random() < 0.85 else int(rng.integers(33, 60))
    m = int(rng.integers(1, 3))
    n = k + m
    L = int(rng.choice([1024, 4096, 4096 + 5, 12 * 1024, 65536, 1000, 48])) if rng.random() < 0.7 \
        else int(rng.integers(1, 30000))
    B = int(rng.integers(1, max(2, min(200, (48 << 20) // (n * L)))))
    aligned = rng.random() < 0.7
    gap = int(16 + (-L) % 16) if aligned else int(rng.integers(0, 9))
    off = 0 if aligned else int(rng.integers(1, 16))
    pitch = L + gap
    case = f"case {c}: k={k} m={m} L={L} B={B} gap={gap} offset={off} items~{B * ((L + 1023) // 1024)}"
    t = torch.empty(B * n * pitch + 64, dtype=torch.uint8).pin_memory()
    a = t.numpy()
    a[:] = rng.integers(0, 256, a.size, dtype=np.uint8)
    before = a.copy()
    view = np.lib.stride_tricks.as_strided(a[off:], (B, n, L), (n * pitch, pitch, 1))
    ref = np.ascontiguousarray(view).copy()
    ref[:, k:] = 0
    assert oracle.encode_strided(ref.reshape(-1), k, m, L, B, L, n * L) == 0
    base = t.data_ptr() + off
    strips = [[[(base + (s * n + j) * pitch, L)] for j in range(n)] for s in range(B)]
    ctx = ec.Ctx()
    try:
        ctx.set_host_pointers(True)
        for s in range(B):
            assert ctx.encode_sg(k, m, strips[s], L) == 0, case
        ctx.flush()
        ctx.synchronize()
        if not (view == ref).all():
            print("ENCODE MISMATCH", case, flush=True)
            sys.exit(1)
        fails = []
        for s in range(B):
            f = sorted(rng.choice(n, int(rng.integers(1, m + 1)), replace=False).tolist())
            fails.append(f)
            for j in f:
                view[s, j] = 0x5A
        for s in range(B):
            assert ctx.reconstruct_sg(k, m, strips[s], L, fails[s]) == 0, case
        ctx.flush()
        ctx.synchronize()
        if not (view == ref).all():
            print("RECONSTRUCT MISMATCH", case, flush=True)
            sys.exit(1)
        # nothing outside the strips was written
        chk = a.copy()
        np.lib.stride_tricks.as_strided(chk[off:], (B, n, L), (n * pitch, pitch, 1))[:] = 0
        np.lib.stride_tricks.as_strided(before[off:], (B, n, L), (n * pitch, pitch, 1))[:] = 0
        if not (chk == before).all():
            print("WROTE OUTSIDE THE STRIPS", case, flush=True)
            sys.exit(1)
    finally:
        ctx.close()
    if (c + 1) % 25 == 0:
        print(f"{c + 1} cases ok (last: {case})", flush=True)
print(f"host ctx soak: {cases} random cases bit-exact against the oracle")

import sys, time, json
import numpy as np
sys.path.insert(0, "draid-spdk_amd")
import torch
import draid_ec as ec
ec.lib()
torch.cuda.init()
for n, L in ((3, 65536), (3, 4096), (10, 65536), (10, 4096), (5, 65536)):
    a = [np.random.randint(0, 256, L, dtype=np.uint8) for _ in range(n)]
    ptrs = [x.ctypes.data for x in a]
    pin = [torch.from_numpy(x.copy()).pin_memory() for x in a]
    pptrs = [x.data_ptr() for x in pin]
    res = {}
    for name, p in (("pageable", ptrs), ("pinned", pptrs)):
        f = (lambda: ec.xor_gen(p, L)) if n in (3, 5) else (lambda: ec.pq_gen(p, L))
        f()
        ts = []
        for _ in range(300):
            t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
        res[name] = round(float(np.median(ts)) * 1e6, 1)
    print(json.dumps({"vects": n, "len": L, **res}), flush=True)

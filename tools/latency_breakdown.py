import sys, time, numpy as np, torch
sys.path.insert(0, '/root/repo/draid-spdk_amd'); sys.path.insert(0, '/root/repo')
import draid_ec as ec
dev = torch.device('cuda', 0)
k, L = 8, 65536; n = k + 2
b = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev)
table = torch.tensor([b[j].data_ptr() for j in range(n)], dtype=torch.int64, device=dev)
batch = ec.make_batch(k, 2, L, 1, table)
s = ec.stream_create()
for i in range(50):
    ec.encode(batch, s)
    while ec.stream_query(s) != 0: pass
t0 = time.perf_counter()
for i in range(2000): ec.stream_query(s)
print('idle stream_query us', (time.perf_counter() - t0) / 2000 * 1e6)
launch = []; polls = []; tot = []
for i in range(300):
    t0 = time.perf_counter()
    ec.encode(batch, s)
    t1 = time.perf_counter()
    np_ = 0
    while ec.stream_query(s) != 0: np_ += 1
    t2 = time.perf_counter()
    launch.append(t1 - t0); polls.append(np_); tot.append(t2 - t0)
print('launch us p50', np.median(launch) * 1e6, 'total p50', np.median(tot) * 1e6, 'polls p50', np.median(polls))
# same with torch's own tiny kernel for comparison
x = torch.zeros(16, device=dev)
st = torch.cuda.Stream(dev)
tt = []
with torch.cuda.stream(st):
    for i in range(300):
        t0 = time.perf_counter()
        x.add_(1)
        while not st.query(): pass
        tt.append(time.perf_counter() - t0)
print('torch add_ + query p50 us', np.median(tt[20:]) * 1e6)

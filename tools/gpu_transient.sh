# Start-up transient of the reconstruct kernel: per-launch durations next to a
# shader-clock probe (tools/probe/transient_probe.hip), and the per-dispatch
# kernel trace of the driver's own bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/transient
mkdir -p $out
export LD_LIBRARY_PATH=$PWD/draid-spdk_amd:$LD_LIBRARY_PATH
echo "probe 8+2 x 64 KiB" && timeout -k 10 120 tools/probe/transient_probe 8 2 64 4096 30 > $out/probe_8p2_64k.jsonl || exit 1
echo "probe 16+2 x 256 KiB" && timeout -k 10 120 tools/probe/transient_probe 16 2 256 512 30 > $out/probe_16p2_256k.jsonl || exit 1
echo "bench (driver command)" && timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_w5.json || exit 1
cd /tmp && export TMPDIR=/tmp
echo "kernel trace of the driver command" && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$out/trace -o w5 -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/bench_w5_traced.json || exit 1
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, json
f = glob.glob('gpurun_out/transient/trace/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
out = {}
for r in rows:
    n = r['Kernel_Name']
    key = 'encode' if 'k_encode' in n else 'reconstruct' if 'k_reconstruct' in n else None
    if key:
        out.setdefault(key, []).append((int(r['Start_Timestamp']), int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
res = {k: [d / 1000.0 for _, d in sorted(v)] for k, v in out.items()}
json.dump(res, open('gpurun_out/transient/per_dispatch_us.json', 'w'))
for k, v in res.items():
    print(k, ' '.join(f'{x:.0f}' for x in v[:30]))
PY
python3 - <<'PY'
import json
for f in ('probe_8p2_64k', 'probe_16p2_256k'):
    for line in open(f'gpurun_out/transient/{f}.jsonl'):
        d = json.loads(line)
        s = d['steps']
        print(f, d['phase'])
        print('  probe_us ', ' '.join(f'{x[0]*1e3:.0f}' for x in s[:16]))
        print('  enc_us   ', ' '.join(f'{x[1]*1e3:.0f}' for x in s[:16]))
        print('  rec_us   ', ' '.join(f'{x[2]*1e3:.0f}' for x in s[:16]))
        print('  cyc/wall ', ' '.join(f'{x[3]/max(1,x[4]):.1f}' for x in s[:16]))
PY

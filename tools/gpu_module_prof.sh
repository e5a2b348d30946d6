# Kernel trace of the raid module bench over null base bdevs (RAID6 8+2 x 64 KiB, qd 32):
# how long the small launches' kernels run, and the gaps between them on the stream.
# Build first: make -C tests/spdk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/modprof; mkdir -p gpurun_out/modprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/modprof -o run -- tests/spdk/build/spdk_raid_module_bench 6 10 64 ${QD:-32} 1 null > gpurun_out/modprof/log.txt 2>&1 || { tail gpurun_out/modprof/log.txt; exit 1; }
tail -6 gpurun_out/modprof/log.txt | cut -c1-300
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/modprof/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = collections.defaultdict(list)
for r in rows:
    by[r['Kernel_Name'][:60]].append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
for k, v in by.items():
    v.sort()
    dur = sorted(e - s for s, e in v)
    gaps = sorted(v[i + 1][0] - v[i][1] for i in range(len(v) - 1))
    print(k, 'n', len(v), 'dur_us p50 %.1f p90 %.1f' % (dur[len(dur)//2]/1e3, dur[len(dur)*9//10]/1e3),
          'gap_us p50 %.1f p90 %.1f' % (gaps[len(gaps)//2]/1e3, gaps[len(gaps)*9//10]/1e3) if gaps else '')
PY

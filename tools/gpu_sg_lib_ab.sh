#!/bin/bash
# A/B of the scatter-gather context between whole library builds inside one GPU
# call: sg_bench (4096 RAID6 8+2 stripes; 64 KiB, 4 KiB and 1 KiB iovecs) with
# LD_LIBRARY_PATH pointing at each build in turn, interleaved rounds.
# usage: gpu_sg_lib_ab.sh "<name>=<dir holding libdraid_ec.so> ..." [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
libs="$1"; rounds="${2:-3}"
mkdir -p gpurun_out
out=gpurun_out/sg_lib_ab.jsonl
rm -f $out
for round in $(seq 1 $rounds); do
  for iov in 65536 4096 1024; do
    for nl in $libs; do
      n=${nl%%=*}; d=${nl#*=}
      LD_LIBRARY_PATH=$PWD/$d:$LD_LIBRARY_PATH timeout -k 10 120 tools/c/sg_bench $iov 4096 10 0 0 | sed "s/^{/{\"lib\": \"$n\", \"round\": $round, /" >> $out || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/sg_lib_ab.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r['iov_bytes'], r['op'], r['lib'])].append(r)
for key in sorted(agg, key=str):
    rs = agg[key]
    def med(f):
        v = sorted(x[f] for x in rs if f in x); return v[len(v)//2] if v else None
    print(key, {f: med(f) for f in ('walk_us_per_stripe', 'flush_ms', 'gpu_ms', 'wall_ms')})
PY

#!/bin/bash
# Same-box A/B of library builds on the scatter-gather benchmark (tools/c/sg_bench):
#   gpu_upd_ab.sh "<name> ..." rounds [iov_bytes ...]     libraries: draid-spdk_amd/libvar/<name>/
# Prints the GPU window (ms per 4096 stripes) of each op per library, round by round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
names="$1"; rounds=${2:-2}; shift 2
iovs="${*:-65536}"
: > gpurun_out/upd_ab.jsonl
for r in $(seq $rounds); do
  for n in $names; do
    for iov in $iovs; do
      LD_LIBRARY_PATH=$PWD/draid-spdk_amd/libvar/$n timeout -k 10 120 tools/c/sg_bench $iov 4096 10 > gpurun_out/upd_ab_one.log || exit 1
      python3 - $n $r >> gpurun_out/upd_ab.jsonl <<'PY'
import json, sys
for l in open('gpurun_out/upd_ab_one.log'):
    if l.startswith('{'):
        d = json.loads(l); d['lib'] = sys.argv[1]; d['round'] = int(sys.argv[2]); print(json.dumps(d))
PY
    done
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open('gpurun_out/upd_ab.jsonl'):
    d = json.loads(l); agg[(d['iov_bytes'], d['op'], d['lib'])].append(d['gpu_ms'])
for k in sorted(agg): print(*k, ' '.join(f'{x:.3f}' for x in agg[k]))
PY

#!/bin/bash
# gf_vect_mul throughput per library build: gpu_gfv_ab.sh "<name> ..." (draid-spdk_amd/libvar/<name>/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
: > gpurun_out/gfv_ab.jsonl
for r in 1 2; do
  for n in $1; do
    DRAID_EC_LIB=$PWD/draid-spdk_amd/libvar/$n/libdraid_ec.so timeout -k 10 120 python3 tools/gf_vect_mul_bench.py > gpurun_out/gfv_one.log || exit 1
    python3 - $n >> gpurun_out/gfv_ab.jsonl <<'PY'
import json, sys
for l in open('gpurun_out/gfv_one.log'):
    d = json.loads(l); d['lib'] = sys.argv[1]; print(json.dumps(d))
PY
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open('gpurun_out/gfv_ab.jsonl'):
    d = json.loads(l); agg[(d['lib'], d['mib'])].append(d['hbm_gb_s'])
for k in sorted(agg): print(*k, agg[k])
PY

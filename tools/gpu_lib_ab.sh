#!/bin/bash
# A/B of whole library builds inside one GPU call: bench.py (the driver's command)
# with DRAID_EC_LIB pointing at each build in turn, interleaved rounds.
# usage: gpu_lib_ab.sh "<name>=<path> ..." [rounds] [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
libs="$1"; rounds="${2:-2}"; shift 2
out=gpurun_out/lib_ab.jsonl
mkdir -p gpurun_out; : > $out
for r in $(seq 1 $rounds); do
  for nl in $libs; do
    n=${nl%%=*}; l=${nl#*=}
    DRAID_EC_LIB=$PWD/$l timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -5 gpurun_out/ab_$n.err; exit 1; }
    python3 - "$n" "$r" gpurun_out/ab_$n.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); b = d['breakdown']
print(json.dumps({"lib": sys.argv[1], "round": int(sys.argv[2]), "config": d['config']['name'], "value": d['value'], "enc_ms": b['encode_ms'], "enc_med": b['encode_ms_median'], "rec_ms": b['reconstruct_ms'], "rec_med": b['reconstruct_ms_median'], "verified": d['verified_roundtrip']}))
PY
    tail -1 $out
  done
done

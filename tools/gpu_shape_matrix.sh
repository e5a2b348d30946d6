#!/bin/bash
# Occupancy study: bench.py --shape over library builds (DRAID_EC_LIB) x stripe shapes.
# usage: gpu_shape_matrix.sh "<lib names under draid-spdk_amd/libx>" "<shapes>" out.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
libs="$1"; shapes="$2"; out="gpurun_out/$3"
mkdir -p gpurun_out; : > $out
for sh in $shapes; do
  for n in $libs; do
    DRAID_EC_LIB=$PWD/draid-spdk_amd/libx/$n/libdraid_ec.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --shape $sh > gpurun_out/m.json 2> gpurun_out/m.err || { tail -5 gpurun_out/m.err; exit 1; }
    python3 - "$n" "$sh" >> $out <<'PY'
import json, sys
d = json.loads(open('gpurun_out/m.json').read().strip().splitlines()[-1]); b = d['breakdown']
print(json.dumps({"lib": sys.argv[1], "shape": sys.argv[2], "value": d['value'], "enc_ms": b['encode_ms'], "rec_ms": b['reconstruct_ms'], "enc_gbs": b['encode_hbm_gb_s'], "rec_gbs": b['reconstruct_hbm_gb_s'], "verified": d['verified_roundtrip']}))
PY
    tail -1 $out
  done
done

#!/bin/bash
# Shader-sequencer counters of the bench's two kernels for one library build:
#   gpu_sq.sh <tag> <lib path> [bench args]
# One --pmc pass (at most 8 SQ counters; SQ_COUNTERS replaces the default set), its own
# run, no trace domains.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; lib=$2; shift 2
O=gpurun_out/sq_$tag; rm -rf $O; mkdir -p $O
export DRAID_EC_LIB=$PWD/$lib
C=${SQ_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY}
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-verify "$@" > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 - $O $tag <<'PY'
import csv, sys, glob, collections, json
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    name = 'reconstruct' if 'k_reconstruct' in k else 'encode' if 'k_encode' in k else None
    if name:
        agg[(name, r['Counter_Name'])].append(float(r['Counter_Value']))
out = collections.defaultdict(dict)
for (n, c), v in agg.items():
    out[n][c] = sum(v) / len(v)
json.dump(out, open(f'{sys.argv[1]}/summary.json', 'w'), indent=1)
for n, d in out.items():
    print(sys.argv[2], n, ' '.join(f"{c}={v:.3g}" for c, v in sorted(d.items())))
PY

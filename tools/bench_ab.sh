# A/B of kernel variants through bench.py itself (lab build, built beforehand):
# V = list of variants (enc | rec << 8), interleaved over R rounds per config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V=${V:-9 0}
R=${R:-2}
CFGS=${CFGS:-raid6_8p2_64k}
out=gpurun_out/bench_ab.jsonl
: > $out
for c in $CFGS; do
  for r in $(seq $R); do
    for v in $V; do
      timeout -k 10 120 python bench.py --config $c --variant $v --no-cpu-baseline --no-verify >> $out 2> gpurun_out/bench_ab.err || { tail gpurun_out/bench_ab.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$out').read().splitlines()[-1]); b=d['breakdown']; print('$c', 'v=$v', b['encode_hbm_gb_s'], b['reconstruct_hbm_gb_s'], d['value'])"
    done
  done
done

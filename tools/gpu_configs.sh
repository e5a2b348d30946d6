#!/bin/bash
# For each BASELINE config: bench line, rocprofv3 kernel trace + stats, and HBM
# traffic from separate --pmc FETCH_SIZE / WRITE_SIZE passes.  Stops at the first
# failing GPU step.  Usage: bash tools/gpu_configs.sh [config ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFGS=${@:-raid6_8p2_64k raid5_4p1_64k raid6_8p2_128k_single raid6_16p2_256k_dual}
for c in $CFGS; do
  O=gpurun_out/cfg_$c
  rm -rf $O; mkdir -p $O
  B="python3 bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-verify"
  echo "== $c bench $(date +%T)"
  timeout -k 10 300 python3 bench.py --config $c --cpu-seconds 5 > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
  tail -1 $O/bench.log
  echo "== $c trace $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
  echo "== $c pmc $(date +%T)"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || { tail $O/pmc_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || { tail $O/pmc_write.log; exit 1; }
  python3 tools/collect_pmc.py trace $O/trace $O/trace_summary.json > /dev/null
  python3 tools/collect_pmc.py pmc $O/pmc_fetch $O/pmc_write $c $O/pmc_$c.json > /dev/null
  python3 - "$O" "$c" <<'PY'
import json, sys
o, c = sys.argv[1], sys.argv[2]
p = json.load(open(f"{o}/pmc_{c}.json"))
t = json.load(open(f"{o}/trace_summary.json"))
for kind in ("encode", "reconstruct"):
    tt = [v for v in t.values() if v["kind"] == kind]
    print(kind, "avg_us", round(tt[0]["avg_us"], 1) if tt else None,
          "hbm_bytes", p.get(f"{kind}_hbm_bytes_per_launch"))
PY
done
echo "== done $(date +%T)"

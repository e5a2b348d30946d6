#!/bin/bash
# Full GPU pass: parity tests, smoke, bench, rocprofv3 kernel trace + stats, and
# HBM traffic from two separate --pmc passes (FETCH_SIZE, WRITE_SIZE).
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify"
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
step bench
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log
step trace
rm -rf $O/prof_trace $O/pmc_fetch $O/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- $B > $O/prof_trace.log 2>&1 || { tail $O/prof_trace.log; exit 1; }
step pmc_fetch
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || { tail $O/pmc_fetch.log; exit 1; }
step pmc_write
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || { tail $O/pmc_write.log; exit 1; }
python3 tools/collect_pmc.py trace $O/prof_trace $O/trace_summary.json > /dev/null
python3 tools/collect_pmc.py pmc $O/pmc_fetch $O/pmc_write raid6_8p2_64k $O/pmc_raid6_8p2_64k.json | head -40
step done

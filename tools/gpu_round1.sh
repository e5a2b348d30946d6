#!/bin/bash
# First GPU pass: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -q -m gpu --maxfail=5 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
echo "== bench"; date
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
echo "== rocprof"; date
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > gpurun_out/prof.log 2>&1 || exit $?
find gpurun_out/prof -name '*stats*' | head
date

#!/bin/bash
# Round check on the GPU box: parity tests (verbose, per-test timeout), the
# allocation-free entry point's test while it is still uncollected, smoke, the
# transient probe and the bench exactly as the driver runs it.  Stops at the
# first failing GPU step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread $PYTEST_EXTRA > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ -f tests/wip_no_alloc.py ]; then
  timeout -k 10 300 python -u -m pytest tests/wip_no_alloc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_wip.log 2>&1 || { tail -40 gpurun_out/pytest_wip.log; exit 1; }
  tail -3 gpurun_out/pytest_wip.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
if [ -x tools/probe/transient_probe ]; then
  timeout -k 10 120 tools/probe/transient_probe 8 2 64 4096 30 > gpurun_out/transient_probe.jsonl || exit 1
  python3 - <<'PY'
import json
for line in open('gpurun_out/transient_probe.jsonl'):
    d = json.loads(line); s = d['steps']
    print(d['phase'], 'rec_us', ' '.join(f'{x[2]*1e3:.0f}' for x in s[:14]), '| GHz', ' '.join(f'{x[3]/max(1,x[4])/10:.1f}' for x in s[:14]))
PY
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { tail gpurun_out/bench_driver.log; exit 1; }
tail -1 gpurun_out/bench_driver.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-900

#!/bin/bash
# Quick end-to-end check: parity tests, smoke, headline bench, one lab sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ "${LAB:-0}" = 1 ]; then
  make -s -C draid-spdk_amd -j8 lab || exit 1
  timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 64 --stripes 4096 --layouts stripe_major --variants 0,10 --rounds 3 --out gpurun_out/sweep_check.json > gpurun_out/sweep_check.log 2>&1 || { tail gpurun_out/sweep_check.log; exit 1; }
  grep -E "^(enc|rec)" gpurun_out/sweep_check.log
fi

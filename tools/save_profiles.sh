#!/bin/bash
# Copy tools/gpu_configs.sh results from gpurun_out/ into profiles/<round>/ and
# refresh profiles/pmc_<config>.json (the per-launch HBM traffic bench.py reports).
R=${1:-r01}
cd "$(dirname "$0")/.."
for d in gpurun_out/cfg_*; do
  c=${d#gpurun_out/cfg_}
  mkdir -p profiles/$R/$c
  grep '^{' $d/bench.log | tail -1 > profiles/$R/$c/bench.json
  cp $d/trace_summary.json profiles/$R/$c/trace_summary.json
  cp $d/trace/run_kernel_stats.csv profiles/$R/$c/kernel_stats.csv
  cp $d/pmc_$c.json profiles/$R/$c/pmc_$c.json
  cp $d/pmc_$c.json profiles/pmc_$c.json
done

#!/bin/bash
# Width matrix of the shipped library: bench.py --shape for every RAID6 width
# 2..32 (dual failure) and a set of RAID5 widths (single failure), 64 KiB
# strips, stripe counts sized to about 2.5 GiB per launch.
# Result: gpurun_out/lib_ab_shapes.jsonl (one line per shape).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
shapes=""
for k in $(seq 2 32); do
  s=$(( 40960 / (k + 2) / 64 * 64 )); shapes="$shapes $k,2,64,$s,dual"
done
for k in 2 3 4 5 6 8 9 12 16 20 24 27 32; do
  s=$(( 40960 / (k + 1) / 64 * 64 )); shapes="$shapes $k,1,64,$s,single"
done
bash tools/gpu_lib_ab_shapes.sh "fin=draid-spdk_amd/libdraid_ec.so" 1 "$shapes"

#!/bin/bash
# Per-TCC-channel request counts of the encode / reconstruct kernels: is the load
# balanced over the memory channels?  rocprofv3 JSON keeps one record per counter
# instance (XCD x channel); tools/channel_balance.py reduces it.
# usage: gpu_channels.sh <config> [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
cfg=${1:-raid6_16p2_256k_dual}; shift
out=$PWD/gpurun_out/channels_$cfg
rm -rf $out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for c in TCC_EA0_RDREQ TCC_EA0_WRREQ; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format json -d $out/$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 4 --warmup 2 --no-cpu-baseline --no-verify "$@" > $out/$c.log 2>&1 || { tail -5 $out/$c.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
ls -la $out/*/ | head; python3 tools/channel_balance.py $out > $out/summary.json && cat $out/summary.json | head -60

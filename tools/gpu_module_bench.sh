# The raid module under bdevperf-shaped load (tests/spdk/bench_raid_module.c):
# RAM base bdevs (every strip copied, like the malloc bdev) and null base bdevs (no
# copies: the module itself), queue depths 32 and 128, with the plain build for the
# rates and the profiling build for the per-request breakdown.
# Build first, here: make -C tests/spdk.   Output: gpurun_out/module_bench.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
O=gpurun_out/module_bench.jsonl
: > $O
SEC=${SEC:-2}
for shape in "6 10 64" "5 5 64" "6 18 256"; do
  for qd in 32 128; do
    for mode in ram null; do
      echo "== raid$shape qd $qd $mode"
      timeout -k 10 120 $B/spdk_raid_module_bench $shape $qd $SEC $mode | sed 's/^{/{"build": "plain", /' >> $O || exit 1
      timeout -k 10 120 $B/spdk_raid_module_bench_prof $shape $qd $SEC $mode | sed 's/^{/{"build": "prof", /' >> $O || exit 1
    done
  done
done
# deeper queues over a larger per-channel request pool: launches of 64 and 128 requests
for r in 128 256; do
  echo "== raid6 10 64 qd $((r * 2)) null, $r requests per channel"
  DRAID_RAID_REQUESTS=$r timeout -k 10 120 $B/spdk_raid_module_bench 6 10 64 $((r * 2)) $SEC null \
      | sed "s/^{/{\"build\": \"plain\", \"requests_per_channel\": $r, /" >> $O || exit 1
  DRAID_RAID_REQUESTS=$r timeout -k 10 120 $B/spdk_raid_module_bench_prof 6 10 64 $((r * 2)) $SEC null \
      | sed "s/^{/{\"build\": \"prof\", \"requests_per_channel\": $r, /" >> $O || exit 1
done
wc -l $O

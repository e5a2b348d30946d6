# The four-thread module harness (simulated threads, OS threads, hot-remove) several
# times over on one box: its OS-thread part is timing dependent, so a failure that
# shows once in N runs shows here.  Stops at the first failing run.
# Build first, here: make -C tests/spdk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
N=${1:-6}
for i in $(seq 1 $N); do
  for t in spdk_raid_threads_test spdk_raid_hotremove_test; do
    timeout -k 10 240 $B/$t > gpurun_out/soak_$t.log 2>&1 || { tail -30 gpurun_out/soak_$t.log; echo "FAILED $t run $i"; exit 1; }
  done
  echo "run $i ok: $(grep -c '^ok' gpurun_out/soak_spdk_raid_threads_test.log) + $(grep -c '^ok' gpurun_out/soak_spdk_raid_hotremove_test.log) checks"
done
echo "module soak: $N runs clean"

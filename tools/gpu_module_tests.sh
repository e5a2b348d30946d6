# The raid module harnesses on the MI355X: the single-thread array checks, the
# four-thread interleaving / OS-thread / hot-remove test, and the hot-remove with the
# redirect compiled into the framework.  Build first, here: make -C tests/spdk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
for t in spdk_raid_threads_test spdk_raid_hotremove_test spdk_raid_module_test; do
    echo "== $t"
    timeout -k 10 240 $B/$t > gpurun_out/$t.log 2>&1 || { tail -30 gpurun_out/$t.log; echo "FAILED $t"; exit 1; }
    tail -12 gpurun_out/$t.log
done
echo "module tests: ok"

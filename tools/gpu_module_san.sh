# The raid module, the reference's bdev_raid.c and the runtime stand-in under
# ASan + UBSan (make -C tests/spdk san) on the MI355X.  Host code only is
# instrumented; libdraid_ec.so stays as built.  Build first, here.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
export ASAN_OPTIONS=detect_leaks=0:quarantine_size_mb=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
L=gpurun_out/spdk_module_asan.log
: > $L
for t in spdk_raid_module_test_asan spdk_raid_threads_test_asan spdk_raid_hotremove_test_asan; do
    echo "== $t" >> $L
    timeout -k 10 400 $B/$t >> $L 2>&1 || { tail -40 $L; echo "FAILED $t"; exit 1; }
done
grep -c "AddressSanitizer\|runtime error" $L && { grep -n "AddressSanitizer\|runtime error" $L | head; exit 1; }
grep "^ok \|array checks" $L | tail -20
echo "asan/ubsan: clean"

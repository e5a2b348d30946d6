# C harness (incl. the disk-rebuild test) and the rebuild throughput tool.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 tests/c/test_draid_raid > gpurun_out/c_harness.log 2>&1 || { tail -30 gpurun_out/c_harness.log; exit 1; }
tail -6 gpurun_out/c_harness.log
: > gpurun_out/rebuild.jsonl
for args in "8 64 4" "8 128 4" "16 256 4"; do
  timeout -k 10 300 tools/c/rebuild_bench $args 5 >> gpurun_out/rebuild.jsonl 2> gpurun_out/rebuild.err || { cat gpurun_out/rebuild.err; exit 1; }
done
cat gpurun_out/rebuild.jsonl

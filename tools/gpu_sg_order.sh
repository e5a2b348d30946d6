# Context address ordering: sg tests, then sg_bench with stripes queued in order,
# shuffled (reordered by the flush), and shuffled with the reordering disabled.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py tests/test_c_harness.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_sg.log 2>&1 || { tail -30 gpurun_out/pytest_sg.log; exit 1; }
tail -1 gpurun_out/pytest_sg.log
rm -f gpurun_out/sg_order.jsonl
for iov in 65536 4096; do
  timeout -k 10 120 tools/c/sg_bench $iov 4096 10 0 >> gpurun_out/sg_order.jsonl || exit 1
  timeout -k 10 120 tools/c/sg_bench $iov 4096 10 1 >> gpurun_out/sg_order.jsonl || exit 1
  DRAID_EC_CTX_ADDRESS_ORDER=0 timeout -k 10 120 tools/c/sg_bench $iov 4096 10 1 | sed 's/"shuffled": 1/"shuffled": 1, "address_order": 0/' >> gpurun_out/sg_order.jsonl || exit 1
done
cat gpurun_out/sg_order.jsonl

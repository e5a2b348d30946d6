# sg tests + C harness, then sg_bench host walk cost at 64 KiB / 4 KiB / 1 KiB iovecs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_rmw.py tests/test_c_harness.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_sg.log 2>&1 || { tail -30 gpurun_out/pytest_sg.log; exit 1; }
tail -1 gpurun_out/pytest_sg.log
rm -f gpurun_out/sg_walk.jsonl
for iov in 65536 4096 1024; do
  timeout -k 10 120 tools/c/sg_bench $iov 4096 10 >> gpurun_out/sg_walk.jsonl || exit 1
done

# Context autoflush: the sg tests, then sg_bench wall time with autoflush off / on
# (64 KiB and 4 KiB iovecs, stripes queued in address order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_sg.log 2>&1 || { tail -30 gpurun_out/pytest_sg.log; exit 1; }
tail -1 gpurun_out/pytest_sg.log
rm -f gpurun_out/sg_autoflush.jsonl
for iov in 65536 4096; do
  for af in 0 256 1024 4096; do
    timeout -k 10 120 tools/c/sg_bench $iov 4096 10 0 $af >> gpurun_out/sg_autoflush.jsonl || exit 1
  done
done

# sg_bench with small flushes (autoflush 256 / 1024 at 64 KiB, 4096 at 4 KiB) and the
# whole-batch flush; sg tests first.  (Used for the same-stream descriptor DMA A/B.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py tests/test_c_harness.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_sg.log 2>&1 || { tail -30 gpurun_out/pytest_sg.log; exit 1; }
tail -1 gpurun_out/pytest_sg.log
rm -f gpurun_out/sg_autoflush2.jsonl
for a in "65536 0" "65536 256" "65536 1024" "4096 0" "4096 4096"; do
  set -- $a
  timeout -k 10 120 tools/c/sg_bench $1 4096 10 0 $2 >> gpurun_out/sg_autoflush2.jsonl || exit 1
done

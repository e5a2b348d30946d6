set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ctx_order.py tests/test_gpu_sg.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_ctx.log 2>&1 || { tail -60 gpurun_out/pytest_ctx.log; exit 1; }
tail -3 gpurun_out/pytest_ctx.log
bash tools/gpu_sg_ahead.sh

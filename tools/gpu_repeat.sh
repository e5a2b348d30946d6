# The GPU suite three times in a row (flakiness check; stops at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:randomly --timeout 240 --timeout-method thread > gpurun_out/pytest_rep$i.log 2>&1 || { tail -30 gpurun_out/pytest_rep$i.log; exit 1; }
  tail -1 gpurun_out/pytest_rep$i.log
done

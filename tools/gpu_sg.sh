set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
make -s -C tools/c
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
rm -f gpurun_out/sg_bench.log
for iov in 65536 4096 1024; do timeout -k 10 120 tools/c/sg_bench $iov 4096 10 >> gpurun_out/sg_bench.log 2>&1 || exit 1; done
export TMPDIR=/tmp
rm -rf gpurun_out/sg_trace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/sg_trace -o run -- tools/c/sg_bench 4096 4096 10 > gpurun_out/sg_trace.log 2>&1 || exit 1
cat gpurun_out/sg_bench.log

# BASELINE config 1 on one box: the CPU harness (isa-l xor_gen restatement on one
# core) next to the GPU-engine harness (tools/c/bdevperf_gpu, built beforehand).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
# (the registered-memory test skips, with the runtime's error, where hipHostRegister is
# refused; bdevperf_gpu then takes its buffers from the pinned allocator and says so)
timeout -k 10 120 python -u -m pytest tests/test_gpu_host.py -x -q -rs -k registered --timeout 60 --timeout-method thread > gpurun_out/pytest_registered.log 2>&1 || { tail -30 gpurun_out/pytest_registered.log; exit 1; }
tail -3 gpurun_out/pytest_registered.log
for q in 32 1; do
  QD=$q SECONDS_RUN=${SECS:-10} timeout -k 10 120 python tools/config1_cpu.py > gpurun_out/config1_cpu_q$q.log 2>&1 || { tail gpurun_out/config1_cpu_q$q.log; exit 1; }
  tail -1 gpurun_out/config1_cpu_q$q.log
  cp gpurun_out/config1_cpu.json gpurun_out/config1_cpu_q$q.json
done
: > gpurun_out/config1_gpu.jsonl
for qg in "1 1" "32 1" "32 2" "32 4" "128 4"; do
  set -- $qg
  timeout -k 10 120 tools/c/bdevperf_gpu ${SECS:-10} $1 $2 >> gpurun_out/config1_gpu.jsonl 2> gpurun_out/config1_gpu.err || { cat gpurun_out/config1_gpu.err; exit 1; }
  tail -1 gpurun_out/config1_gpu.jsonl
done

# Secondary measurements after a kernel change: scatter-gather context path,
# host-buffer (PCIe) path, per-call latency, config-4 strong scaling at N=1, and
# a 2-rank rehearsal of the multi-GPU bench (gloo timing collectives, both ranks
# on the one GPU).  Stops at the first failing GPU step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/sg_bench.log
for iov in 65536 4096 1024; do timeout -k 10 120 tools/c/sg_bench $iov 4096 10 >> gpurun_out/sg_bench.log 2>&1 || { cat gpurun_out/sg_bench.log; exit 1; }; done
cat gpurun_out/sg_bench.log
timeout -k 10 300 python tools/host_path_bench.py > gpurun_out/host_path.log 2>&1 || { tail gpurun_out/host_path.log; exit 1; }
grep '^{' gpurun_out/host_path.log | head -4
timeout -k 10 300 python tools/latency.py > gpurun_out/latency.log 2>&1 || { tail gpurun_out/latency.log; exit 1; }
timeout -k 10 300 python bench.py --config raid6_8p2_128k_single --strong --no-cpu-baseline > gpurun_out/strong_n1.log 2>&1 || { tail gpurun_out/strong_n1.log; exit 1; }
tail -1 gpurun_out/strong_n1.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu-baseline > gpurun_out/rehearse_n2.log 2>&1 || { tail -20 gpurun_out/rehearse_n2.log; exit 1; }
grep '^{' gpurun_out/rehearse_n2.log | cut -c1-400

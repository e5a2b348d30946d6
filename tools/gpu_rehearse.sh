set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu-baseline > gpurun_out/rehearse_n2.log 2>&1 || { tail -20 gpurun_out/rehearse_n2.log; exit 1; }
grep '^{' gpurun_out/rehearse_n2.log | cut -c1-300
grep -o '"verified_roundtrip": [a-z]*' gpurun_out/rehearse_n2.log

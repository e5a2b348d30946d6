set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
make -s -C draid-spdk_amd -j8 lab || exit 1
timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -q -x -k "reconstruct or roundtrip or unaligned" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 64 --stripes 4096 --failures dual --layouts stripe_major --variants ${VARIANTS:-0,14,15} --rounds 7 --out gpurun_out/sweep_diag.json > gpurun_out/swd.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/swd.log

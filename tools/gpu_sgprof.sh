set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/sgp; mkdir -p gpurun_out/sgp
for iov in 65536 4096 1024; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sgp/i$iov -o run -- tools/c/sg_bench $iov 4096 10 > gpurun_out/sgp/log_$iov.txt 2>&1 || exit 1
done

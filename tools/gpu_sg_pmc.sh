# HBM traffic of the scatter-gather kernels (sg_bench, 4096 stripes of RAID6 8+2 x 64 KiB,
# 1 rep): rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/sgpmc
rm -rf $O; mkdir -p $O
for iov in 65536 4096; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$iov -o run -- tools/c/sg_bench $iov 4096 1 > $O/f$iov.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$iov -o run -- tools/c/sg_bench $iov 4096 1 > $O/w$iov.log 2>&1 || exit 1
done
ls $O

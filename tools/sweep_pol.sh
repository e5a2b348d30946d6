# Cache policy of the one-wave kernels: nt loads / nt stores on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
make -s -C draid-spdk_amd -j8 lab || exit 1
V=${V:-0,21,22,23}
timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 64 --stripes 4096 --failures dual --layouts stripe_major --variants $V --out gpurun_out/sweepp_8p2_64k.json > gpurun_out/swp1.log 2>&1 || exit 1
timeout -k 10 300 python tools/sweep.py --k 16 --strip-kib 256 --stripes 512 --failures dual --layouts stripe_major --variants $V --out gpurun_out/sweepp_16p2_256k.json > gpurun_out/swp2.log 2>&1 || exit 1
timeout -k 10 300 python tools/sweep.py --k 4 --strip-kib 64 --stripes 4096 --failures single --layouts stripe_major --variants $V --out gpurun_out/sweepp_4p1_64k.json > gpurun_out/swp3.log 2>&1 || exit 1

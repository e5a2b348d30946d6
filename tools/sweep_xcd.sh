# XCD-aware item order and workgroup size vs strip size (stripe-major / strip-major).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
make -s -C draid-spdk_amd -j8 lab || exit 1
V=${V:-0,9,18,19,20}
timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 64 --stripes 4096 --failures dual --layouts stripe_major --variants $V --out gpurun_out/sweepx_8p2_64k.json > gpurun_out/swx1.log 2>&1 || exit 1
timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 128 --stripes 4096 --failures single --layouts stripe_major,strip_major --variants $V --out gpurun_out/sweepx_8p2_128k.json > gpurun_out/swx2.log 2>&1 || exit 1
timeout -k 10 300 python tools/sweep.py --k 16 --strip-kib 256 --stripes 512 --failures dual --layouts stripe_major,strip_major --variants $V --out gpurun_out/sweepx_16p2_256k.json > gpurun_out/swx3.log 2>&1 || exit 1
timeout -k 10 300 python tools/sweep.py --k 4 --strip-kib 64 --stripes 4096 --failures single --layouts stripe_major --variants $V --out gpurun_out/sweepx_4p1_64k.json > gpurun_out/swx4.log 2>&1 || exit 1

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
make -s -C draid-spdk_amd -j8 lab || exit 1
L=stripe_major,stripe_major_gap4096,stripe_major_gap65536,strip_major
V=0,1,2,4,10,11,12
timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 128 --stripes 4096 --failures single --layouts $L --variants $V --out gpurun_out/sweep_8p2_128k.json > gpurun_out/sw1.log 2>&1 || exit 1
timeout -k 10 300 python tools/sweep.py --k 16 --strip-kib 256 --stripes 512 --failures dual --layouts $L --variants $V --out gpurun_out/sweep_16p2_256k.json > gpurun_out/sw2.log 2>&1 || exit 1
timeout -k 10 300 python tools/sweep.py --k 4 --strip-kib 64 --stripes 4096 --failures single --layouts $L --variants $V --out gpurun_out/sweep_4p1_64k.json > gpurun_out/sw3.log 2>&1 || exit 1
for f in 1 2 3; do echo "--- sw$f"; grep -v amdgpu gpurun_out/sw$f.log | head -12; grep -v amdgpu gpurun_out/sw$f.log | grep '^rec' | head -8; done

# Cache policy of the one-wave kernels (lab build, built beforehand on the CPU
# side: make -C draid-spdk_amd lab): nt loads / nt stores on and off, and the
# explicit sc0 / sc1 / nt bits through buffer instructions (variants 24-33).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V=${V:-0,24,25,26,27,28,29,30,31,32,33}
R=${ROUNDS:-3}
run() {  # name k strip_kib stripes failures
  timeout -k 10 300 python tools/sweep.py --k $2 --strip-kib $3 --stripes $4 --failures $5 --layouts stripe_major --variants $V --rounds $R --out gpurun_out/sweepp_$1.json > gpurun_out/swp_$1.log 2>&1 || { tail gpurun_out/swp_$1.log; exit 1; }
  grep -E "^(verify|enc|rec)" gpurun_out/swp_$1.log
}
run 8p2_64k 8 64 4096 dual && run 4p1_64k 4 64 4096 single && run 8p2_128k 8 128 4096 single && run 16p2_256k 16 256 512 dual

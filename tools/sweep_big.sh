# Large-strip shapes (8+2 x 128 KiB, 16+2 x 256 KiB): item order, lanes and
# vectors per lane (lab build, built beforehand).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V=${V:-0,9,4,18,19,20,2,10}
R=${ROUNDS:-3}
L=${LAYOUTS:-stripe_major}
run() {  # name k strip_kib stripes failures
  timeout -k 10 300 python tools/sweep.py --k $2 --strip-kib $3 --stripes $4 --failures $5 --layouts $L --variants $V --rounds $R --out gpurun_out/sweepb_$1.json > gpurun_out/swb_$1.log 2>&1 || { tail gpurun_out/swb_$1.log; exit 1; }
  grep -E "^(verify|enc|rec)" gpurun_out/swb_$1.log
}
run 16p2_256k 16 256 512 dual && run 8p2_128k 8 128 4096 single

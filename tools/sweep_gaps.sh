# Stripe-major placement with a gap between strips (lab build): does a skew
# between strips help the large-strip shapes?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=${LAYOUTS:-stripe_major,stripe_major_gap8192,stripe_major_gap16384,stripe_major_gap65536,stripe_major_gap131072,strip_major}
run() {  # name k strip_kib stripes failures
  timeout -k 10 300 python tools/sweep.py --k $2 --strip-kib $3 --stripes $4 --failures $5 --layouts $L --variants 0 --rounds 3 --out gpurun_out/sweepg_$1.json > gpurun_out/swg_$1.log 2>&1 || { tail gpurun_out/swg_$1.log; exit 1; }
  grep -E "^(enc|rec)" gpurun_out/swg_$1.log
}
run 16p2_256k 16 256 512 dual && run 8p2_128k 8 128 2048 single

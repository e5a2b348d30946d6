# Stripe-major vs strip-major placement at every BASELINE shape (lab build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V=${V:-0,9,2,38}
R=${ROUNDS:-3}
run() {  # name k strip_kib stripes failures
  timeout -k 10 300 python tools/sweep.py --k $2 --strip-kib $3 --stripes $4 --failures $5 --layouts stripe_major,strip_major --variants $V --rounds $R --out gpurun_out/sweepl_$1.json > gpurun_out/swl_$1.log 2>&1 || { tail gpurun_out/swl_$1.log; exit 1; }
  grep -E "^(enc|rec)" gpurun_out/swl_$1.log
}
run 8p2_64k 8 64 4096 dual && run 4p1_64k 4 64 4096 single && run 8p2_128k 8 128 4096 single && run 16p2_256k 16 256 512 dual

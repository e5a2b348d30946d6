# Parity placement and slot order at every BASELINE shape (lab build, production variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V=${V:-0}
R=${ROUNDS:-3}
L=${LAYOUTS:-stripe_major,parity_apart,stripe_shuffled,strip_major}
run() {  # name k strip_kib stripes failures
  timeout -k 10 300 python tools/sweep.py --k $2 --strip-kib $3 --stripes $4 --failures $5 --layouts $L --variants $V --rounds $R --out gpurun_out/sweepl2_$1.json > gpurun_out/swl2_$1.log 2>&1 || { tail gpurun_out/swl2_$1.log; exit 1; }
  grep -E "^(enc|rec)" gpurun_out/swl2_$1.log
}
run 8p2_64k 8 64 4096 dual && run 4p1_64k 4 64 4096 single && run 8p2_128k 8 128 4096 single && run 16p2_256k 16 256 512 dual

# Reconstruct time vs how failure pairs are spread over the batch (lab build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for o in random sorted fixed; do
  timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 64 --stripes 4096 --failures dual --layouts stripe_major --variants 0,9 --rounds 3 --fail-order $o --out gpurun_out/sweepf_$o.json > gpurun_out/swf_$o.log 2>&1 || { tail gpurun_out/swf_$o.log; exit 1; }
  echo "== $o"; grep -E "^(verify|rec)" gpurun_out/swf_$o.log
done

# Stripe-to-slot order: shuffled slots, and shuffled runs of G slots (lab build, production variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/sweep.py --k 8 --strip-kib 64 --stripes 4096 --failures dual --layouts stripe_major,stripe_shuffled,stripe_shuffled_g2,stripe_shuffled_g4,stripe_shuffled_g16,stripe_shuffled_g64,stripe_shuffled_g256 --variants 0 --rounds 3 --out gpurun_out/sweeps_8p2_64k.json > gpurun_out/sws_8p2_64k.log 2>&1 || { tail gpurun_out/sws_8p2_64k.log; exit 1; }
grep -E "^(enc|rec)" gpurun_out/sws_8p2_64k.log

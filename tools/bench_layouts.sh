# bench.py at every BASELINE config in both stripe placements (verified round trips).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/bench_layouts.jsonl
: > $out
for c in raid6_8p2_64k raid5_4p1_64k raid6_8p2_128k_single raid6_16p2_256k_dual; do
  for l in stripe_major strip_major; do
    timeout -k 10 120 python bench.py --config $c --layout $l --no-cpu-baseline >> $out 2> gpurun_out/bench_layouts.err || { tail gpurun_out/bench_layouts.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out').read().splitlines()[-1]); b=d['breakdown']; print('$c $l', d['value'], b['encode_hbm_gb_s'], b['reconstruct_hbm_gb_s'], d['verified_roundtrip'])"
  done
done

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B=tests/spdk/build
O=gpurun_out/module_throttle_levels.jsonl
: > $O
for round in 1 2; do
for shape in "6 10 64" "6 18 256"; do
  for qd in 32 64 128 256; do
    for lds in 0 57344 131072; do
      DRAID_RAID_REQUESTS=128 DRAID_EC_THROTTLE_LDS=$lds timeout -k 10 120 $B/spdk_raid_module_bench $shape $qd 1.5 null | sed "s/^{/{\"lds\": $lds, \"round\": $round, /" >> $O || exit 1
    done
  done
done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/module_throttle_levels.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    if r['job'] in ('full_stripe_read',): continue
    agg[(r['n'], r['qd'], r['job'], r['lds'])].append(round(r['mib_s']))
for k in sorted(set(k[:3] for k in agg), key=str):
    print(k, ' | '.join(f"{l//1024}K: {agg[k+(l,)]}" for l in (0, 57344, 131072)))
PY

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B=tests/spdk/build
O=gpurun_out/module_slots.jsonl
: > $O
for round in 1 2; do
for g in 1 2 4; do
  for shape in "6 10 64" "5 5 64"; do
    for qd in 32 128; do
      DRAID_RAID_GPUS=$g timeout -k 10 120 $B/spdk_raid_module_bench $shape $qd 2 null | sed "s/^{/{\"slots\": $g, \"round\": $round, /" >> $O || exit 1
    done
  done
done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/module_slots.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r['n'], r['qd'], r['job'], r['slots'])].append(round(r['mib_s']))
for k in sorted(agg, key=str): print(k, agg[k])
PY

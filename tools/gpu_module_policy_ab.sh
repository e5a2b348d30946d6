# The module bench built with other launch policies (RG_MAX_INFLIGHT launches in flight
# per GPU, a launch at most 1 / RG_TAKE_DIV of the busy requests; variants built by hand
# into tests/spdk/build/bench_<name>) beside the product's, interleaved, null disks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
O=gpurun_out/module_policy_ab.jsonl
: > $O
for round in 1 2; do
  for qd in 32 128; do
    for v in spdk_raid_module_bench $1; do
      timeout -k 10 120 $B/$v 6 10 64 $qd ${SEC:-1.5} null | sed "s/^{/{\"variant\": \"$v\", \"round\": $round, /" >> $O || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/module_policy_ab.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r['qd'], r['job'], r['variant'])].append(r['mib_s'])
for k in sorted(agg, key=str):
    print(k, [round(x) for x in agg[k]])
PY

# The raid module over null and RAM base bdevs with host-resident launches throttled
# to one item per CU (the default) against full occupancy (DRAID_EC_THROTTLE_LDS=0),
# interleaved.  Build first: make -C tests/spdk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
O=gpurun_out/module_throttle_ab.jsonl
: > $O
SEC=${SEC:-2}
for round in 1 2; do
  for shape in "6 10 64" "5 5 64" "6 18 256"; do
    for qd in 32 128; do
      for mode in null ram; do
        for t in on off; do
          if [ $t = off ]; then export DRAID_EC_THROTTLE_LDS=0; else unset DRAID_EC_THROTTLE_LDS; fi
          timeout -k 10 120 $B/spdk_raid_module_bench $shape $qd $SEC $mode \
              | sed "s/^{/{\"throttle\": \"$t\", \"round\": $round, /" >> $O || exit 1
        done
      done
    done
  done
done
unset DRAID_EC_THROTTLE_LDS
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/module_throttle_ab.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r['n'], r['strip_kib'], r['qd'], r['base_bdevs'], r['job'], r['throttle'])].append(r['mib_s'])
for k in sorted(set(k[:5] for k in agg), key=str):
    a, b = agg[k + ('on',)], agg[k + ('off',)]
    print(k, 'throttled', [round(x) for x in a], 'full', [round(x) for x in b], '%+.1f%%' % ((sum(a) / len(a)) / (sum(b) / len(b)) * 100 - 100))
PY

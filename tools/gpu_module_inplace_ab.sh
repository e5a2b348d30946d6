# The raid module over null base bdevs with its launches' descriptors read in place
# from pinned memory (the default for launches of up to 256 segments) against uploaded
# first (DRAID_EC_CTX_INPLACE_LIMIT=0), interleaved, plain build for the rates and
# profiling build for the reactor's time per request.  Build first: make -C tests/spdk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
O=gpurun_out/module_inplace_ab.jsonl
: > $O
SEC=${SEC:-2}
for round in 1 2; do
  for shape in "6 10 64" "5 5 64" "6 18 256"; do
    for qd in 32 128; do
      for mode in null ram; do
        for n in 256 0; do
          DRAID_EC_CTX_INPLACE_LIMIT=$n timeout -k 10 120 $B/spdk_raid_module_bench $shape $qd $SEC $mode \
              | sed "s/^{/{\"build\": \"plain\", \"inplace\": $n, \"round\": $round, /" >> $O || exit 1
        done
      done
    done
  done
done
for n in 256 0; do
  DRAID_EC_CTX_INPLACE_LIMIT=$n timeout -k 10 120 $B/spdk_raid_module_bench_prof 6 10 64 32 $SEC null \
      | sed "s/^{/{\"build\": \"prof\", \"inplace\": $n, \"round\": 1, /" >> $O || exit 1
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/module_inplace_ab.jsonl')]
print(sorted(rows[0].keys()))
agg = collections.defaultdict(list)
for r in rows:
    if r['build'] != 'plain':
        continue
    agg[(r.get('level'), r.get('n'), r.get('strip_kib'), r.get('qd'), r.get('mode', r.get('disks')), r.get('job'), r['inplace'])].append(r.get('mib_s'))
for k in sorted(agg, key=str):
    print(k, agg[k])
PY

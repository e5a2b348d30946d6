# The raid module over null and RAM base bdevs with two builds of the library, interleaved:
# usage gpu_module_lib_ab.sh <old.so> <new.so> ["qd ..."].  The harness binaries find the
# library through their run path, so each run first copies its build over
# draid-spdk_amd/libdraid_ec.so (on the GPU box's scratch copy of the tree); the new one is
# back in place at the end.  Build first: make -C tests/spdk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tests/spdk/build
O=gpurun_out/module_lib_ab.jsonl
OLD=$1; NEW=$2; QDS=${3:-"32 128"}
cp $NEW gpurun_out/lib_new.so && cp $OLD gpurun_out/lib_old.so || exit 1
: > $O
SEC=${SEC:-2}
for round in 1 2; do
  for shape in "6 10 64" "5 5 64" "6 18 256"; do
    for qd in $QDS; do
      for mode in null ram; do
        for t in old new; do
          cp gpurun_out/lib_$t.so draid-spdk_amd/libdraid_ec.so
          timeout -k 10 120 $B/spdk_raid_module_bench $shape $qd $SEC $mode \
              | sed "s/^{/{\"lib\": \"$t\", \"round\": $round, /" >> $O || { cp gpurun_out/lib_new.so draid-spdk_amd/libdraid_ec.so; exit 1; }
        done
      done
    done
  done
done
cp gpurun_out/lib_new.so draid-spdk_amd/libdraid_ec.so
rm -f gpurun_out/lib_new.so gpurun_out/lib_old.so
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/module_lib_ab.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r['n'], r['strip_kib'], r['qd'], r['base_bdevs'], r['job'], r['lib'])].append(r['mib_s'])
for k in sorted(set(k[:5] for k in agg), key=str):
    a, b = agg[k + ('new',)], agg[k + ('old',)]
    print(k, 'new', [round(x) for x in a], 'old', [round(x) for x in b], '%+.1f%%' % ((sum(a) / len(a)) / (sum(b) / len(b)) * 100 - 100))
PY

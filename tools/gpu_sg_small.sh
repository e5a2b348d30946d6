# Small flushes (a poller's batch): sg_bench at 1..1024 stripes per flush with the
# descriptors read in place from pinned memory up to N segments (the default N, and
# N = 0: always uploaded), interleaved rounds.  Build first: make -C draid-spdk_amd &&
# make -C tools/c.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/sg_small_ab.jsonl
rm -f $out
for round in 1 2 3; do
  for b in ${STRIPES_LIST:-2 8 16 32 64 128 256 1024}; do
    for n in ${INPLACE_LIST:-1000000 0}; do
      DRAID_EC_CTX_INPLACE_LIMIT=$n timeout -k 10 120 tools/c/sg_bench ${IOV:-65536} $b 300 0 0 | sed "s/^{/{\"inplace\": $n, \"round\": $round, /" >> $out || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/sg_small_ab.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r['stripes'], r['op'], r['inplace'])].append(r)
for key in sorted(agg):
    rs = agg[key]
    def med(f):
        v = sorted(x[f] for x in rs); return v[len(v)//2]
    print(key, 'flush_us %.1f gpu_us %.1f wall_us %.1f' % (med('flush_ms')*1e3, med('gpu_ms')*1e3, med('wall_ms')*1e3))
PY

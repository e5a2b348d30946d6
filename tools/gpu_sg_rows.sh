# A/B of the context's row format inside one GPU call: compact rows (base pointer +
# 32-bit offsets, the default) against rows of 64-bit pointers (DRAID_EC_CTX_ROWS=64),
# sg_bench over 4096 RAID6 8+2 stripes at 64 KiB, 4 KiB and 1 KiB iovecs, interleaved
# rounds.  Build first, here: make -C draid-spdk_amd && make -C tools/c (sg_bench).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/sg_rows_ab.jsonl
rm -f $out
for round in 1 2 3; do
  for iov in 65536 4096 1024; do
    for rows in compact 64; do
      if [ $rows = 64 ]; then export DRAID_EC_CTX_ROWS=64; else unset DRAID_EC_CTX_ROWS; fi
      timeout -k 10 120 tools/c/sg_bench $iov 4096 10 0 0 | sed "s/^{/{\"rows\": \"$rows\", \"round\": $round, /" >> $out || exit 1
    done
  done
done
unset DRAID_EC_CTX_ROWS
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/sg_rows_ab.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r.get('iov_bytes', r.get('iov')), r['op'], r['rows'])].append(r)
for key in sorted(agg, key=str):
    rs = agg[key]
    def med(f):
        v = sorted(x[f] for x in rs if f in x); return v[len(v)//2] if v else None
    print(key, {f: med(f) for f in rs[0] if isinstance(rs[0][f], float)})
PY

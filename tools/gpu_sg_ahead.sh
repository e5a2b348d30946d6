# A/B of the context's early descriptor uploads inside one GPU call: pieces uploaded
# from inside the queueing calls (the default) against uploads at flush time only
# (DRAID_EC_CTX_STAGE_AHEAD=0), sg_bench over 4096 RAID6 8+2 stripes at 64 KiB, 4 KiB
# and 1 KiB iovecs, interleaved rounds.  Build first, here: make -C draid-spdk_amd &&
# make -C tools/c (sg_bench).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/sg_ahead_ab.jsonl
rm -f $out
for round in 1 2 3; do
  for iov in 65536 4096 1024; do
    for ahead in 1 0; do
      if [ $ahead = 0 ]; then export DRAID_EC_CTX_STAGE_AHEAD=0; else unset DRAID_EC_CTX_STAGE_AHEAD; fi
      timeout -k 10 120 tools/c/sg_bench $iov 4096 10 0 0 | sed "s/^{/{\"ahead\": $ahead, \"round\": $round, /" >> $out || exit 1
    done
  done
done
unset DRAID_EC_CTX_STAGE_AHEAD
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/sg_ahead_ab.jsonl')]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r['iov_bytes'], r['op'], r['ahead'])].append(r)
for key in sorted(agg, key=str):
    rs = agg[key]
    def med(f):
        v = sorted(x[f] for x in rs if f in x); return v[len(v)//2] if v else None
    print(key, {f: med(f) for f in ('walk_us_per_stripe', 'flush_ms', 'gpu_ms', 'wall_ms')})
PY

#!/bin/bash
# gpu_lib_ab.sh over several shapes: usage gpu_lib_ab_shapes.sh "<name>=<lib> ..." rounds "K,M,KIB,STRIPES,FAIL ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
libs="$1"; rounds="$2"; shapes="$3"
: > gpurun_out/lib_ab_shapes.jsonl
for sh in $shapes; do
  bash tools/gpu_lib_ab.sh "$libs" "$rounds" --shape "$sh" > /dev/null || exit 1
  python3 - "$sh" >> gpurun_out/lib_ab_shapes.jsonl <<'PY'
import json, sys
for l in open('gpurun_out/lib_ab.jsonl'):
    d = json.loads(l); d['shape'] = sys.argv[1]; print(json.dumps(d))
PY
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open('gpurun_out/lib_ab_shapes.jsonl')]
agg = collections.defaultdict(list)
for r in rows: agg[(r['shape'], r['lib'])].append(r)
for (sh, lib), rs in agg.items():
    print(sh, lib, 'value', ' '.join(f"{r['value']:.0f}" for r in rs), 'enc', ' '.join(f"{r['enc_med']*1e3:.1f}" for r in rs), 'rec', ' '.join(f"{r['rec_med']*1e3:.1f}" for r in rs))
PY

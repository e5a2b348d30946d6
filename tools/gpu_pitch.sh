#!/bin/bash
# Stripe-pitch / strip-pitch skew study: bench.py --shape with padded pitches.
# usage: gpu_pitch.sh "<shapes>" "<stripe pads>" "<strip pads>" out.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
shapes="$1"; spads="$2"; tpads="$3"; out="gpurun_out/$4"
mkdir -p gpurun_out; : > $out
for sh in $shapes; do
  for tp in $tpads; do
    for sp in $spads; do
      timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --shape $sh --stripe-pad $sp --strip-pad $tp > gpurun_out/p.json 2> gpurun_out/p.err || { tail -5 gpurun_out/p.err; exit 1; }
      python3 - "$sh" "$sp" "$tp" >> $out <<'PY'
import json, sys
d = json.loads(open('gpurun_out/p.json').read().strip().splitlines()[-1]); b = d['breakdown']
print(json.dumps({"shape": sys.argv[1], "stripe_pad": int(sys.argv[2]), "strip_pad": int(sys.argv[3]), "value": d['value'], "enc_ms": b['encode_ms'], "rec_ms": b['reconstruct_ms'], "enc_gbs": b['encode_hbm_gb_s'], "rec_gbs": b['reconstruct_hbm_gb_s'], "verified": d['verified_roundtrip']}))
PY
      tail -1 $out
    done
  done
done

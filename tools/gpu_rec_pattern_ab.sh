# tools/rec_pair_pattern.py over library variants built by tools/build_variants.sh
# (usage: gpu_rec_pattern_ab.sh "name ..."; "base" is the product library).  The variants
# travel only while ./draid-spdk_amd/libvar is commented out in .gpurunignore.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/rec_pattern_ab.jsonl
for round in 1 2; do
  for v in $1; do
    lib=draid-spdk_amd/libvar/$v/libdraid_ec.so
    [ "$v" = base ] && lib=draid-spdk_amd/libdraid_ec.so
    DRAID_EC_LIB=$PWD/$lib timeout -k 10 120 python -u tools/rec_pair_pattern.py > gpurun_out/rec_pattern_one.json || exit 1
    python3 - "$v" "$round" >> gpurun_out/rec_pattern_ab.jsonl <<'PY'
import json, sys
d = json.load(open('gpurun_out/rec_pattern_one.json')); d['lib'] = sys.argv[1]; d['round'] = int(sys.argv[2]); print(json.dumps(d))
PY
  done
done
cat gpurun_out/rec_pattern_ab.jsonl

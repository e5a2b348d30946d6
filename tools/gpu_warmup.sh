set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 10 20 40; do
timeout -k 10 200 python bench.py --warmup $w --no-cpu-baseline > gpurun_out/wu_$w.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/wu_$w.log').read().strip().splitlines()[-1]); b=d['breakdown']; print($w, d['value'], b['encode_ms'], b['encode_ms_median'], b['reconstruct_ms'], b['reconstruct_ms_median'])"
done

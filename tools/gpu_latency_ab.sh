# A/B of tools/latency.py: the library under draid-spdk_amd/ab_old/ (selected with
# DRAID_EC_LIB) against the current one, two interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/lat_ab.jsonl
for r in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then export DRAID_EC_LIB=draid-spdk_amd/ab_old/libdraid_ec.so; else unset DRAID_EC_LIB; fi
    timeout -k 10 120 python tools/latency.py > gpurun_out/lat_$lib.log 2>&1 || { tail gpurun_out/lat_$lib.log; exit 1; }
    sed "s/^{/{\"lib\": \"$lib\", /" gpurun_out/lat_$lib.log | grep '^{' >> gpurun_out/lat_ab.jsonl
  done
done
cat gpurun_out/lat_ab.jsonl

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
make -s -C tools/c
for iov in 65536 4096; do timeout -k 10 120 tools/c/sg_bench $iov 4096 10 >> gpurun_out/sg_bench.log 2>&1 || exit 1; done
ldconfig -p | grep -i isal > gpurun_out/isal_probe.txt 2>&1; ls /usr/lib/x86_64-linux-gnu /usr/local/lib 2>/dev/null | grep -i isal >> gpurun_out/isal_probe.txt; lscpu | head -20 >> gpurun_out/isal_probe.txt
bash tools/gpu_configs.sh

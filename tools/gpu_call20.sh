set -e
make -s -C tools/probe
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python3 tools/probe_stripes.py > gpurun_out/probe_stripes.log 2>&1
timeout -k 10 300 python3 tools/host_path_bench.py > gpurun_out/host_path.log 2>&1
timeout -k 10 200 python3 bench.py --config raid6_8p2_64k --stripes 8192 --no-cpu-baseline --steps 20 > gpurun_out/b64_8192.log 2>&1
timeout -k 10 200 python3 bench.py --config raid6_8p2_128k_single --stripes 2048 --no-cpu-baseline --steps 20 > gpurun_out/b128_2048.log 2>&1
timeout -k 10 200 python3 bench.py --config raid6_8p2_128k_single --no-cpu-baseline --steps 20 > gpurun_out/b128_4096.log 2>&1

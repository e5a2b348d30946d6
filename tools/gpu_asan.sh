# Host code of the library under AddressSanitizer on the MI355X (tests/c/Makefile
# san-gpu: host side instrumented, kernels not): the C harness end to end, and the
# scatter-gather context with stripes queued out of order (reordered by default at
# 64 KiB, and forced with DRAID_EC_CTX_ADDRESS_ORDER=2 at 4 KiB and 1 KiB iovecs), then
# in queue order.
# Build first, here: make -C tests/c san-gpu (the binaries are git-ignored but travel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
# quarantine_size_mb=0: ROCm's ASan runtime otherwise recycles runtime-owned
# chunks after the HSA runtime has unloaded (a CHECK failure at process exit)
export ASAN_OPTIONS=detect_leaks=0:quarantine_size_mb=0
L=gpurun_out/asan.log
: > $L
timeout -k 10 300 tests/c/test_draid_raid_asan_gpu >> $L 2>&1 || { tail -40 $L; exit 1; }
timeout -k 10 120 tests/c/sg_bench_asan_gpu 65536 512 2 1 >> $L 2>&1 || { tail -40 $L; exit 1; }
DRAID_EC_CTX_ADDRESS_ORDER=2 timeout -k 10 120 tests/c/sg_bench_asan_gpu 4096 256 2 1 >> $L 2>&1 || { tail -40 $L; exit 1; }
DRAID_EC_CTX_ADDRESS_ORDER=2 timeout -k 10 120 tests/c/sg_bench_asan_gpu 1024 64 2 1 >> $L 2>&1 || { tail -40 $L; exit 1; }
# queue order kept: pointer tables DMA'd from the context's pinned storage, with and
# without autoflush (the next batch walked while earlier copies are in flight)
timeout -k 10 120 tests/c/sg_bench_asan_gpu 1024 256 3 0 >> $L 2>&1 || { tail -40 $L; exit 1; }
timeout -k 10 120 tests/c/sg_bench_asan_gpu 4096 512 3 0 1024 >> $L 2>&1 || { tail -40 $L; exit 1; }
# enough small segments for descriptor pieces uploaded ahead of the flush (three per
# batch at 1 KiB iovecs x 1024 stripes), alone and with autoflush launching between them
timeout -k 10 180 tests/c/sg_bench_asan_gpu 1024 1024 2 0 >> $L 2>&1 || { tail -40 $L; exit 1; }
timeout -k 10 180 tests/c/sg_bench_asan_gpu 1024 1024 2 0 30000 >> $L 2>&1 || { tail -40 $L; exit 1; }
# one batch of more descriptor pieces than the context has ring slots (28 over 16): slots of
# the batch's own earlier pieces are waited for and used again inside the one flush
DRAID_EC_CTX_STAGE_AHEAD=0 timeout -k 10 240 tests/c/sg_bench_asan_gpu 1024 8192 1 0 >> $L 2>&1 || { tail -40 $L; exit 1; }
timeout -k 10 240 tests/c/sg_bench_asan_gpu 1024 8192 1 0 >> $L 2>&1 || { tail -40 $L; exit 1; }
# pageable memory: the pinned bounce arena and the device arena of the isa-l-shaped calls,
# and host stripes bounced through pinned buffers by the calling thread
timeout -k 10 300 tests/c/test_pageable_asan_gpu >> $L 2>&1 || { tail -40 $L; exit 1; }
grep -c "AddressSanitizer" $L && exit 1
grep -c "^PASS" $L
tail -12 $L
echo "asan: clean"

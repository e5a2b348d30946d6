# A/B of the context's descriptor upload: pointer tables DMA'd straight from the
# group's pinned storage (current library) against packing them into a ring
# slot first (the previous ec_ctx.cpp, built beside it into
# draid-spdk_amd/ab_old/ and selected through LD_LIBRARY_PATH, which takes
# precedence over sg_bench's RUNPATH).  GPU tests on the current library first.
# The old library was built here from `git show <previous commit>:draid-spdk_amd/csrc/ec_ctx.cpp`
# with the Makefile's HIPFLAGS, linked against the other build/*.o objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_sg.log 2>&1 || { tail -30 gpurun_out/pytest_sg.log; exit 1; }
tail -1 gpurun_out/pytest_sg.log
out=gpurun_out/sg_direct_ab.jsonl
rm -f $out
for round in 1 2 3; do
  for a in "65536 0" "4096 0" "1024 0" "65536 1024" "4096 4096"; do
    set -- $a
    for lib in old new; do
      if [ $lib = old ]; then pre="env LD_LIBRARY_PATH=draid-spdk_amd/ab_old"; else pre=""; fi
      $pre timeout -k 10 120 tools/c/sg_bench $1 4096 10 0 $2 | sed "s/^{/{\"lib\": \"$lib\", \"autoflush\": $2, /" >> $out || exit 1
    done
  done
done
echo done

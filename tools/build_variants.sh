#!/bin/bash
# Builds whole-library variants for same-box A/B runs (tools/gpu_lib_ab.sh):
#   build_variants.sh name1="-DDRAID_REC_WAVES=8" name2="-DDRAID_ENC_SPLIT=3 -DDRAID_ENC_WAVES=5" ...
# Each variant recompiles csrc/ec_kernels.hip with its flags and links it with the
# product's other objects into draid-spdk_amd/libvar/<name>/libdraid_ec.so (git-ignored; travels to the GPU box).
set -e
cd "$(dirname "$0")/../draid-spdk_amd"
make -s libdraid_ec.so
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops"
OBJS="build/ec_static.o build/ec_api.o build/ec_ctx.o build/ec_host.o build/ec_xlate.o build/ec_mgpu.o build/draid_raid.o build/draid_stripe_cache.o"
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  mkdir -p build/var/$name libvar/$name
  ( $HIPCC $FLAGS $flags -c csrc/ec_kernels.hip -o build/var/$name/ec_kernels.o 2> build/var/$name/build.log &&
    $HIPCC -shared --offload-arch=gfx950 -o libvar/$name/libdraid_ec.so build/var/$name/ec_kernels.o $OBJS ) &
  pids+=($!)
  if [ ${#pids[@]} -ge 6 ]; then wait ${pids[0]}; pids=("${pids[@]:1}"); fi
done
wait
for spec in "$@"; do name=${spec%%=*}; ls -la libvar/$name/libdraid_ec.so; done

#!/bin/bash
# Two counter passes (instruction mix; LDS and issue activity) over the production
# library for the headline and the widest config; summaries land in gpurun_out/sq_*/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=draid-spdk_amd/libdraid_ec.so
for cfg in raid6_8p2_64k raid6_16p2_256k_dual; do
  bash tools/gpu_sq.sh mix_$cfg $L --config $cfg || exit 1
  SQ_COUNTERS="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES" \
    bash tools/gpu_sq.sh lds_$cfg $L --config $cfg || exit 1
done

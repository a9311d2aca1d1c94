#!/bin/bash
# PMC issue / wait anatomy of the level-0 3x3 halo conv (tools/gemm_one.py, id 33 = 128 px x 64 channels, two blocks
# per CU), one counter set per rocprofv3 run (rocprofv3 does not split counters over passes).
#   bash tools/ab/pmc_halo.sh <tag>
set -e
out=gpurun_out/${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  n=$((n + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "conv_halo" -d "$out/pmc_halo_$n" -o run \
    --output-format csv -- python3 tools/gemm_one.py --shape 1,72,96,320,320,3 --algo 33 --split 1 --reps 10 \
    > "$out/pmc_halo_$n.txt" 2>&1
  echo "set $n done"
done

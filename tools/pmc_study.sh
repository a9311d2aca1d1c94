#!/bin/bash
# PMC study of single dc_conv_gemm shapes (tools/gemm_one.py, 20 warm launches each): where the waves'
# cycles go (pass A) and the instruction mix (pass B).  Each pass is its own rocprofv3 run.
# Usage: bash tools/pmc_study.sh <tag>
set -e
tag=${1:-study}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
i=0
while read -r shape algo split; do
  [ -z "$shape" ] && continue
  i=$((i+1))
  for p in A B; do
    ctr=${!p}
    timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex conv_gemm -d $out/s${i}_$p -o run \
      --output-format csv -- python3 tools/gemm_one.py --shape $shape --algo $algo --split $split --reps 20 \
      > $out/s${i}_$p.log 2>&1
  done
  echo "s$i $shape $algo $split" >> $out/index.txt
done <<LIST
1,72,96,320,320,3 13 -3
1,72,96,320,320,3 10 -2
1,72,96,320,320,3 10 1
1,1,6912,320,320,1 13 1
1,18,24,1280,1280,3 3 2
1,1,4096,4096,4096,1 10 1
1,1,4096,4096,4096,1 14 1
LIST
echo "pmc study $tag done"

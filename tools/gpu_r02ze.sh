#!/bin/bash
# r02ze: L2 / L1-to-L2 counters of single dc_conv_gemm shapes on their tuned 64x64 variants (tools/gemm_one.py,
# 20 warm launches each): L2 hit rate and L1 -> L2 read requests, against the operand-fill model of tools/fill_rate.py
set -e
out=gpurun_out/r02ze
mkdir -p $out
export TMPDIR=/tmp
i=0
while read -r shape algo split; do
  [ -z "$shape" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
    --kernel-include-regex conv_gemm -d $out/s${i} -o run --output-format csv -- \
    python3 tools/gemm_one.py --shape $shape --algo $algo --split $split --reps 20 > $out/s${i}.log 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --kernel-include-regex conv_gemm -d $out/t${i} -o run \
    --output-format csv -- python3 tools/gemm_one.py --shape $shape --algo $algo --split $split --reps 20 \
    > $out/t${i}.log 2>&1
  echo "s$i $shape $algo $split" >> $out/index.txt
done <<LIST
1,72,96,320,320,3 13 -3
1,18,24,1280,1280,3 3 2
1,1,6912,320,320,1 13 1
LIST
echo r02ze done

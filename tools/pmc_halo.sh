#!/bin/bash
# SQ counters of one conv shape under a few (algo, split) choices (halo vs im2col), each its own rocprofv3 pass.
# Usage: bash tools/pmc_halo.sh <tag> <shape nb,h,w,cin,cout,k> <algo:split> ...
set -e
tag=$1; shape=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for as in "$@"; do
  a=${as%:*}; sp=${as#*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $out/pmc_${a}_${sp} -o run --output-format csv -- \
    python3 tools/gemm_one.py --shape $shape --algo $a --split $sp --reps 30 > $out/pmc_${a}_${sp}.log 2>&1
  echo "pmc $a:$sp done"
done

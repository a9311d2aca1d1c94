#!/bin/bash
# r02p: cold-cache GEMM tuning of the C4 (batch 1 / 8) and C5 (10-seed ensemble) shapes on top of the
# committed C2 / C3 table
set -e
out=gpurun_out/r02p
mkdir -p $out
DC_TUNE_COLD=1 timeout -k 10 1000 python -u tools/tune_gemm.py --workloads c4:1 c4:8 c5:1 --out $out/tuned_gfx950.json > $out/tune.log 2>&1
echo r02p done

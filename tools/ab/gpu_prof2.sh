#!/bin/bash
# PMC passes of the dominant kernel (conv_gemm) over an eager bench step (4 denoising steps):
# FETCH_SIZE, WRITE_SIZE and the MFMA-busy pass, for one batch size.  Usage: bash tools/ab/gpu_prof2.sh <tag> <batch>
set -e
tag=${1:-run}; batch=${2:-1}
out=gpurun_out/$tag/b$batch
mkdir -p $out
export TMPDIR=/tmp
common="--no-graph --steps 1 --warmup 0 --no-cpu-baseline --denoise-steps 4 --batch $batch"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_gemm -d $out/pmc_fetch -o run \
  --output-format csv -- python3 bench.py $common > $out/pmc_fetch.json 2> $out/pmc_fetch.err
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_gemm -d $out/pmc_write -o run \
  --output-format csv -- python3 bench.py $common > $out/pmc_write.json 2> $out/pmc_write.err
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  --kernel-include-regex conv_gemm -d $out/pmc_mfma -o run \
  --output-format csv -- python3 bench.py $common > $out/pmc_mfma.json 2> $out/pmc_mfma.err
echo "prof2 $tag b$batch done"

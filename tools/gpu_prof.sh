#!/bin/bash
# GPU-box profiling pass for one tag: kernel-trace stats of the C2 bench + the two PMC passes of the
# dominant kernel.  Every GPU step has its own time limit; the script stops at the first failure.
# Usage: bash tools/gpu_prof.sh <tag>
set -e
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/trace_bench.json 2> $out/trace.err
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_gemm -d $out/pmc_fetch -o run \
  --output-format csv -- python3 bench.py --no-graph --steps 1 --warmup 0 --no-cpu-baseline --denoise-steps 4 \
  > $out/pmc_fetch.json 2> $out/pmc_fetch.err
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_gemm -d $out/pmc_write -o run \
  --output-format csv -- python3 bench.py --no-graph --steps 1 --warmup 0 --no-cpu-baseline --denoise-steps 4 \
  > $out/pmc_write.json 2> $out/pmc_write.err
echo "prof $tag done"

#!/bin/bash
# r02g: kernel-trace stats of the C2 bench (current build), C4 sequence at batch 8 per GPU
set -e
out=gpurun_out/r02g
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/trace_bench.json 2> $out/trace.err
timeout -k 10 300 python3 -u bench.py --height 352 --width 1216 --pattern beams --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c4_b8.json 2> $out/bench_c4_b8.err
echo r02g done

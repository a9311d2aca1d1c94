#!/bin/bash
# r02q: C4 b1 / b8 and C5 ensemble bench lines with the C4 / C5 shapes in the tuned table
set -e
out=gpurun_out/r02q
mkdir -p $out
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4.json 2> $out/bench_c4.err
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c4_b8.json 2> $out/bench_c4_b8.err
timeout -k 10 300 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
echo r02q done

#!/bin/bash
# r02l part 2: C3 b8, C4 beams b1 / b8, C5 10-seed ensemble, PMC passes b1 / b8
set -e
out=gpurun_out/r02l
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c3_b8.json 2> $out/bench_c3_b8.err
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4.json 2> $out/bench_c4.err
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c4_b8.json 2> $out/bench_c4_b8.err
timeout -k 10 300 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err
bash tools/gpu_prof2.sh r02l 1
bash tools/gpu_prof2.sh r02l 8
echo r02l part 2 done

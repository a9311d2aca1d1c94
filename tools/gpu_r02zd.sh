#!/bin/bash
# r02zd: C4 (64-beam, batch 1 / 8) and C5 (10-seed ensemble) bench lines on HEAD, C2 once more for the box
set -e
out=gpurun_out/r02zd
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4.json 2> $out/bench_c4.err
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c4_b8.json 2> $out/bench_c4_b8.err
timeout -k 10 300 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err
echo r02zd done

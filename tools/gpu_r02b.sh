#!/bin/bash
# r02b: counter list, GEMM headroom vs hipBLASLt, C4 / C5-ensemble bench lines
set -e
out=gpurun_out/r02b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
timeout -k 10 400 python -u tools/blas_ref.py > $out/blas_ref.txt 2> $out/blas_ref.err
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_c4.json 2> $out/bench_c4.err
timeout -k 10 300 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err
echo r02b done

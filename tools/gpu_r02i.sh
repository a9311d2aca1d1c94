#!/bin/bash
# r02i: GEMM loop: scalar wave index + steady-state wait (conv tests, headroom table, C2 bench)
set -e
out=gpurun_out/r02i
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 200 --timeout-method thread -k "conv or gemm or linear" > $out/kernels.log 2>&1
timeout -k 10 400 python -u tools/blas_ref.py > $out/blas_ref.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
echo r02i done

#!/bin/bash
# r02j: GEMM mainloop software-pipelined by k-half (conv tests, headroom table, C2 + C3 b8 bench)
set -e
out=gpurun_out/r02j
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 200 --timeout-method thread -k "conv or gemm or linear" > $out/kernels.log 2>&1
timeout -k 10 400 python -u tools/blas_ref.py > $out/blas_ref.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
timeout -k 10 300 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c3_b8.json 2> $out/bench_c3_b8.err
echo r02j done

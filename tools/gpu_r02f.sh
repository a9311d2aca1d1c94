#!/bin/bash
# r02f: cross-attention MFMA kernels (tests + timing), GEMM rasterisation A/B (M-major vs auto N-major), C2 bench
set -e
out=gpurun_out/r02f
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "cross or conv" > $out/kernels.log 2>&1
timeout -k 10 120 python -u tools/cross_bench.py > $out/cross_bench.txt 2>&1
DC_GEMM_ORDER=1 timeout -k 10 400 python -u tools/blas_ref.py > $out/blas_ref_mmajor.txt 2>&1
timeout -k 10 400 python -u tools/blas_ref.py > $out/blas_ref_auto.txt 2>&1
DC_GEMM_ORDER=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_c2_mmajor.json 2> $out/bench_c2_mmajor.err
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
echo r02f done

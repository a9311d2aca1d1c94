#!/bin/bash
# r02w: conv_gemm prologue on 32-bit multiply-shift division -- kernel / model / pipeline tests, C2 bench A/B
# against the HEAD library (ab_build/libdcamd_base.so via DC_LIB)
set -e
out=gpurun_out/r02w
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -v --timeout 300 --timeout-method thread > $out/kernel_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -k "parity or replay or sparse_aware or baseline_config" -x -v --timeout 300 --timeout-method thread > $out/pipe_tests.log 2>&1
for i in 1 2; do
  DC_LIB=ab_build/libdcamd_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_base_$i.json 2> $out/bench_base_$i.err
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_new_$i.json 2> $out/bench_new_$i.err
done
echo r02w done

#!/bin/bash
# r02u: GroupNorm finalize inside the statistics launch -- GN kernel tests, pipeline tests, C2 A/B (DC_GN_FUSED)
set -e
out=gpurun_out/r02u
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k groupnorm -v --timeout 300 --timeout-method thread > $out/gn_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_session.py -x -v --timeout 300 --timeout-method thread > $out/pipe_tests.log 2>&1
for i in 1 2; do
  DC_GN_FUSED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_unfused_$i.json 2> $out/bench_unfused_$i.err
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_fused_$i.json 2> $out/bench_fused_$i.err
done
echo r02u done

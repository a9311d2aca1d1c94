#!/bin/bash
# r02zi: weight-stationary narrow convs (DC_CONV_WS=1: 64-row tiles, 8-stage A ring; 2: 128-row tiles, 4 stages) --
# kernel tests and pipeline parity with each, C2 bench A/B (same library, env switch); then the conv PMC passes
set -e
out=gpurun_out/r02zi
mkdir -p $out
export TMPDIR=/tmp
for w in 1 2; do
  DC_CONV_WS=$w timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "conv or linear" -x -v --timeout 300 --timeout-method thread > $out/conv_tests_ws$w.log 2>&1
done
DC_CONV_WS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_models.py -k "parity or replay or taesd or decode" -x -v --timeout 300 --timeout-method thread > $out/pipe_tests_ws1.log 2>&1
for i in 1 2; do
  for w in 0 1 2; do
    DC_CONV_WS=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_ws${w}_$i.json 2> $out/bench_ws${w}_$i.err
  done
done
DC_CONV_WS=1 timeout -k 10 300 python -u tools/conv_breakdown.py > $out/conv_breakdown_ws1.txt 2> $out/conv_breakdown_ws1.err
bash tools/gpu_prof2.sh r02zi 1
bash tools/gpu_prof2.sh r02zi 8
echo r02zi done

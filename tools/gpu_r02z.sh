#!/bin/bash
# r02z: conv output rows by write-through (sc1) stores (DC_CONV_WT=1) -- conv tests and pipeline parity with it
# on, C2 / C3 bench A/B (same library, env switch)
set -e
out=gpurun_out/r02z
mkdir -p $out
export TMPDIR=/tmp
DC_CONV_WT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "conv or linear" -x -v --timeout 300 --timeout-method thread > $out/conv_tests_wt.log 2>&1
DC_CONV_WT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -k "parity or replay" -x -v --timeout 300 --timeout-method thread > $out/pipe_tests_wt.log 2>&1
for i in 1 2; do
  DC_CONV_WT=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_wt0_$i.json 2> $out/bench_wt0_$i.err
  DC_CONV_WT=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_wt1_$i.json 2> $out/bench_wt1_$i.err
done
DC_CONV_WT=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_wt0.json 2> $out/bench_c3_wt0.err
DC_CONV_WT=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_wt1.json 2> $out/bench_c3_wt1.err
echo r02z done

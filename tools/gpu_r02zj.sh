#!/bin/bash
# r02zj: GroupNorm elementwise passes issue their first row's loads ahead of the in-block partial fold (DC_GN_PF,
# default on) -- GN kernel tests and pipeline parity with it, C2 bench A/B (same library, env switch), C3 A/B
set -e
out=gpurun_out/r02zj
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "groupnorm" -x -v --timeout 300 --timeout-method thread > $out/gn_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -k "parity or replay" -x -v --timeout 300 --timeout-method thread > $out/pipe_tests.log 2>&1
for i in 1 2 3; do
  DC_GN_PF=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_pf0_$i.json 2> $out/bench_pf0_$i.err
  DC_GN_PF=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_pf1_$i.json 2> $out/bench_pf1_$i.err
done
DC_GN_PF=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_pf0.json 2> $out/bench_c3_pf0.err
DC_GN_PF=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_pf1.json 2> $out/bench_c3_pf1.err
echo r02zj done

#!/bin/bash
# r02zb: 8-wave (two k-step quads) twins of the 64x64 / 128x64 BK-64 GEMM tiles -- kernel tests of the new algos,
# pipeline parity with DC_CONV_W8=1, C2 / C3 bench A/B (same library, env switch), conv breakdown with it
set -e
out=gpurun_out/r02zb
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "conv or linear or geglu" -x -v --timeout 300 --timeout-method thread > $out/conv_tests.log 2>&1
DC_CONV_W8=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_baseline_configs.py -k "parity or replay or c1 or c2 or c3 or C1 or C2 or C3 or ensemble" -x -v --timeout 300 --timeout-method thread > $out/pipe_tests_w8.log 2>&1
for i in 1 2; do
  DC_CONV_W8=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_w0_$i.json 2> $out/bench_w0_$i.err
  DC_CONV_W8=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_w8_$i.json 2> $out/bench_w8_$i.err
done
DC_CONV_W8=1 timeout -k 10 300 python -u tools/conv_breakdown.py > $out/conv_breakdown_w8.txt 2> $out/conv_breakdown_w8.err
DC_CONV_W8=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_w0.json 2> $out/bench_c3_w0.err
DC_CONV_W8=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_w8.json 2> $out/bench_c3_w8.err
echo r02zb done

#!/bin/bash
# r02v: packed-fp32 softmax arithmetic in the attention kernels -- attention + pipeline tests, attention
# microbench and C2 bench A/B against the HEAD library (ab_build/libdcamd_base.so via DC_LIB)
set -e
out=gpurun_out/r02v
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "attention or cross" -v --timeout 300 --timeout-method thread > $out/attn_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -k "parity or replay or closed_form" -x -v --timeout 300 --timeout-method thread > $out/pipe_tests.log 2>&1
DC_LIB=ab_build/libdcamd_base.so timeout -k 10 120 python -u tools/attn_bench.py > $out/attn_bench_base.txt 2>&1
timeout -k 10 120 python -u tools/attn_bench.py > $out/attn_bench_new.txt 2>&1
for i in 1 2; do
  DC_LIB=ab_build/libdcamd_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_base_$i.json 2> $out/bench_base_$i.err
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_new_$i.json 2> $out/bench_new_$i.err
done
echo r02v done

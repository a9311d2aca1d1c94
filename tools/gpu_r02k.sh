#!/bin/bash
# r02k: attention forward with lazy rescale + MFMA row sums (attention tests, A/B microbench, C2 bench)
set -e
out=gpurun_out/r02k
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 200 --timeout-method thread -k "attention" > $out/attn_tests.log 2>&1
DC_LIB=abtmp/libdcamd_base.so timeout -k 10 200 python -u tools/attn_bench.py > $out/attn_base.txt 2>&1
timeout -k 10 200 python -u tools/attn_bench.py > $out/attn_new.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
echo r02k done

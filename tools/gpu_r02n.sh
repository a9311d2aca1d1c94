#!/bin/bash
# r02n: attention fwd (lazy rescale, fp32 row sums) + delta fused into dQ: attention / session / pipeline tests,
# accuracy vs fp32 SDPA, microbench A/B, C2 bench
set -e
out=gpurun_out/r02n
mkdir -p $out
timeout -k 10 200 python -u tools/attn_acc.py > $out/acc_new.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pipeline.py tests/test_gpu_session.py -v -s --timeout 250 --timeout-method thread -k "attention or vae_original or session or c2 or ensemble" > $out/tests.log 2>&1
DC_LIB=abtmp/libdcamd_base.so timeout -k 10 200 python -u tools/attn_bench.py > $out/attn_base.txt 2>&1
timeout -k 10 200 python -u tools/attn_bench.py > $out/attn_new.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
echo r02n done

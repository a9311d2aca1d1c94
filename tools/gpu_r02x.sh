#!/bin/bash
# r02x: GroupNorm finalize folded into the apply blocks (2 launches per GN at levels 0-1) + one division per
# thread for the channel groups -- GN / pipeline tests, C2 and C3 bench A/B against the previous library
set -e
out=gpurun_out/r02x
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k groupnorm -v --timeout 300 --timeout-method thread > $out/gn_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_session.py -k "parity or replay or sparse_aware or baseline_config or session or native" -x -v --timeout 300 --timeout-method thread > $out/pipe_tests.log 2>&1
for i in 1 2; do
  DC_LIB=ab_build/libdcamd_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_base_$i.json 2> $out/bench_base_$i.err
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_new_$i.json 2> $out/bench_new_$i.err
done
DC_LIB=ab_build/libdcamd_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_base.json 2> $out/bench_c3_base.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_new.json 2> $out/bench_c3_new.err
echo r02x done

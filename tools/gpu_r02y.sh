#!/bin/bash
# r02y: conv 2^31 check fix (linears over > 46341 rows) + GroupNorm finalize folded into the apply blocks:
# full GPU suite, C2 and C3 bench A/B against the conv-fix-only library (ab_build/libdcamd_base.so)
set -e
out=gpurun_out/r02y
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gputest.log 2>&1
for i in 1 2; do
  DC_LIB=ab_build/libdcamd_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_base_$i.json 2> $out/bench_base_$i.err
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_new_$i.json 2> $out/bench_new_$i.err
done
DC_LIB=ab_build/libdcamd_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_base.json 2> $out/bench_c3_base.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 8 --steps 2 > $out/bench_c3_new.json 2> $out/bench_c3_new.err
echo r02y done

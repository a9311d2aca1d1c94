#!/bin/bash
# round 5: GroupNorm in the skinny split-K reduction with batched gathers, C2 A/B by DC_GN_REDUCE (same binary: the
# switch selects launches, no kernel code changes), its unit tests, and the call timeline (sparse setup rewritten)
set -e
out=gpurun_out/r05e
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gn_fused.py -k reduce -m gpu -v -s --timeout 300 \
  --timeout-method thread > "$out/gputest.log" 2>&1
for rep in 1 2 3; do
  for v in 1 0; do
    DC_GN_REDUCE=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$out/c2_red${v}_$rep.json" 2> "$out/c2_red${v}_$rep.err"
  done
done
bash tools/gpu.sh r05e calltrace stepprof

#!/bin/bash
# round 5: GroupNorm in the skinny split-K reduction (tests, C2 A/B by DC_GN_REDUCE), attention before / after (ab/old =
# the tree before the forward's max / sum chains), the FF2 + proj_out fold probe, attention PMC passes
set -e
out=gpurun_out/r05d
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_gn_fused.py tests/test_gpu_models.py tests/test_gpu_session.py -m gpu -v -s --timeout 300 \
  --timeout-method thread > "$out/gputest.log" 2>&1
for rep in 1 2; do
  for v in 1 0; do
    DC_GN_REDUCE=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$out/c2_red${v}_$rep.json" 2> "$out/c2_red${v}_$rep.err"
  done
done
timeout -k 10 300 python -u tools/attn_bench.py > "$out/attn_new.txt" 2>&1
(cd ab/old && timeout -k 10 300 python -u ../../tools/attn_bench.py) > "$out/attn_old.txt" 2>&1
timeout -k 10 300 python -u tools/attn_bench.py > "$out/attn_new2.txt" 2>&1
timeout -k 10 400 python -u tools/fuse_probe.py > "$out/fuse_probe.txt" 2>&1
bash tools/ab/pmc_attn.sh r05d

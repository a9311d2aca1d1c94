#!/bin/bash
# Re-tune the stride-1 3x3 shapes (halo kernel candidates included) with cold caches, then A/B the C2 / C3 bench
# lines old table vs new table on the same box, alternating.  Usage: bash tools/ab/retune_ab.sh <tag>
set -e
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
DC_TUNE_COLD=1 timeout -k 10 1200 python -u tools/tune_gemm.py --retune-3x3 --workloads c2:1 c2:8 c4:1 c4:8 c5:1 \
  --out $out/tuned.json > $out/tune.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_old_$i.json 2> $out/c2_old_$i.err
  DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_new_$i.json 2> $out/c2_new_$i.err
done
timeout -k 10 300 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/c3_old.json 2> $out/c3_old.err
DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline \
  > $out/c3_new.json 2> $out/c3_new.err
echo "retune $tag done"

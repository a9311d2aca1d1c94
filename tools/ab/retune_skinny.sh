#!/bin/bash
# Cold-weight re-tune (DC_TUNE_COLD=2: caches flushed, then the activations read back, the step's state) of the few-pixel shapes (C2 / C4 at batch 1) with the weight-streaming skinny variants as candidates
# (tools/tune_gemm.py --try: the committed choice against the skinny ids only), then A/B the C2 / C4 bench lines old
# table vs new table on the same box, alternating.  Usage: bash tools/ab/retune_skinny.sh <tag>
set -e
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
DC_TUNE_COLD=2 timeout -k 10 900 python -u tools/tune_gemm.py --try ${IDS:-$(seq 43 54)} --workloads ${WL:-c2:1 c4:1} \
  --out $out/tuned.json > $out/tune.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_old_$i.json 2> $out/c2_old_$i.err
  DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_new_$i.json 2> $out/c2_new_$i.err
done
timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --no-cpu-baseline > $out/c4_old.json 2> $out/c4_old.err
DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --no-cpu-baseline \
  > $out/c4_new.json 2> $out/c4_new.err
echo "retune $tag done"

#!/bin/bash
# Full re-tune of every conv shape of the C2 step (all algo ids, all splits: tune_gemm.py --try with every id) in
# the step's cache state -- weights cold, activations warm (DC_TUNE_COLD=2) -- then A/B the C2 bench line old table
# vs new table on the same box, alternating.  Usage: bash tools/retune_warm_act.sh <tag> [workloads...]
set -e
tag=${1:?tag}
shift
wl=${*:-c2:1}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
DC_TUNE_COLD=2 timeout -k 10 1000 python -u tools/tune_gemm.py --try $(seq 1 54) --workloads $wl \
  --out $out/tuned.json > $out/tune.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_old_$i.json 2> $out/c2_old_$i.err
  DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_new_$i.json 2> $out/c2_new_$i.err
done
echo "retune $tag done"

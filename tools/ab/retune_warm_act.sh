#!/bin/bash
# Full re-tune of every conv shape of the given workloads (all algo ids, all splits: tune_gemm.py --try with every
# id) in the step's cache state -- weights cold, activations warm (DC_TUNE_COLD=2) -- then A/B a bench line old table
# vs new table on the same box, alternating.
#   bash tools/ab/retune_warm_act.sh <tag> [workloads] [bench args]     e.g.  r03w8 "c2:8" "--batch 8 --steps 2 --warmup 1"
set -e
tag=${1:?tag}
wl=${2:-c2:1}
bargs=${3:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
nalg=$(python -c "from depth_completion_amd import _lib; print(_lib.load().dc_conv_num_algos())")
# shellcheck disable=SC2086
DC_TUNE_COLD=2 timeout -k 10 1000 python -u tools/tune_gemm.py --try $(seq 1 $nalg) --workloads $wl \
  --out $out/tuned.json > $out/tune.log 2>&1
for i in 1 2; do
  # shellcheck disable=SC2086
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $bargs > $out/old_$i.json 2> $out/old_$i.err
  # shellcheck disable=SC2086
  DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --no-cpu-baseline $bargs > $out/new_$i.json 2> $out/new_$i.err
done
echo "retune $tag done"

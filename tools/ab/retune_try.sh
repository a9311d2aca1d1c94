#!/bin/bash
# Re-time every conv shape of the workloads: its committed choice against the given algo ids only (tune_gemm.py
# --try), in the step's cache state (DC_TUNE_COLD=2: weights cold, activations warm), then A/B bench lines old table
# vs new table on the same box, alternating.
#   bash tools/ab/retune_try.sh <tag> "<algo ids>" [workloads] [bench args]
set -e
tag=${1:?tag}
ids=${2:?algo ids}
wl=${3:-c2:1}
bargs=${4:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
# shellcheck disable=SC2086
DC_TUNE_COLD=2 timeout -k 10 1000 python -u tools/tune_gemm.py --try $ids --workloads $wl \
  --out $out/tuned.json > $out/tune.log 2>&1
for i in 1 2; do
  # shellcheck disable=SC2086
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $bargs > $out/old_$i.json 2> $out/old_$i.err
  # shellcheck disable=SC2086
  DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --no-cpu-baseline $bargs > $out/new_$i.json 2> $out/new_$i.err
done
echo "retune $tag done"

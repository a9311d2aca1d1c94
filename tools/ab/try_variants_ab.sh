#!/bin/bash
# Re-time every shape of the given workloads: the committed choice against the listed algo ids only (cold caches),
# then A/B the C2 (and C3 batch-8) bench lines with the committed vs the new table, alternating.
# Usage: bash tools/ab/try_variants_ab.sh <tag> "<workloads>" <algo ids...>
set -e
tag=${1:?tag}
wls=${2:?workloads}
shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
# shellcheck disable=SC2086
DC_TUNE_COLD=1 timeout -k 10 1200 python -u tools/tune_gemm.py --workloads $wls --try "$@" --out $out/tuned.json \
  > $out/tune.log 2>&1
grep "re-timed shapes changed" $out/tune.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_old_$i.json 2> $out/c2_old_$i.err
  DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_new_$i.json 2> $out/c2_new_$i.err
done
timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/c3_old.json 2> $out/c3_old.err
DC_TUNED=$out/tuned.json timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline \
  > $out/c3_new.json 2> $out/c3_new.err
echo "try $tag done"

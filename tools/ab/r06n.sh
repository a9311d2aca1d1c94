#!/bin/bash
# Round 6 final: the round-5 tree (ab/old, its own library and tuned table) against this tree, alternating on one box:
# C2 three pairs, C3 (batch 8) and C5 (10-seed ensemble) two pairs each.
set -e
out=gpurun_out/r06n
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
for rep in 1 2 3; do
  (cd ab/old && timeout -k 10 300 python -u bench.py --no-cpu-baseline) > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep $(v $out/c2_old_$rep.json) $(v $out/c2_new_$rep.json)"
done
for rep in 1 2; do
  (cd ab/old && timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline) > "$out/c3_old_$rep.json" 2> "$out/c3_old_$rep.err"
  timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_new_$rep.json" 2> "$out/c3_new_$rep.err"
  echo "c3 $rep $(v $out/c3_old_$rep.json) $(v $out/c3_new_$rep.json)"
done
for rep in 1 2; do
  (cd ab/old && timeout -k 10 400 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 \
    --no-cpu-baseline) > "$out/c5_old_$rep.json" 2> "$out/c5_old_$rep.err"
  timeout -k 10 400 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 \
    --no-cpu-baseline > "$out/c5_new_$rep.json" 2> "$out/c5_new_$rep.err"
  echo "c5 $rep $(v $out/c5_old_$rep.json) $(v $out/c5_new_$rep.json)"
done
echo done

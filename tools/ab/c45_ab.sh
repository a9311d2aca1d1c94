#!/bin/bash
# Alternating C4 (KITTI 64-beam) and C5 (10-seed ensemble) bench lines: committed table vs another.
#   bash tools/ab/c45_ab.sh <tag> <pairs> <table>
set -e
out=gpurun_out/${1:?tag}
mkdir -p "$out"
c4() { timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --no-cpu-baseline; }
c5() { timeout -k 10 400 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 --no-cpu-baseline; }
for w in c4 c5; do
  for i in $(seq 1 "${2:?pairs}"); do
    $w > "$out/${w}_a_$i.json" 2> "$out/${w}_a_$i.err"
    DC_TUNED=${3:?table} $w > "$out/${w}_b_$i.json" 2> "$out/${w}_b_$i.err"
    echo "$w $i $(python3 -c "import json;print(json.load(open('$out/${w}_a_$i.json'))['value'], json.load(open('$out/${w}_b_$i.json'))['value'])")"
  done
done

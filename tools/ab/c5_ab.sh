#!/bin/bash
# Alternating C5 (10-seed ensemble) bench lines: committed table vs another.   bash tools/ab/c5_ab.sh <tag> <pairs> <table>
set -e
out=gpurun_out/${1:?tag}
mkdir -p "$out"
c5() { timeout -k 10 400 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 --no-cpu-baseline; }
for i in $(seq 1 "${2:?pairs}"); do
  c5 > "$out/a_$i.json" 2> "$out/a_$i.err"
  DC_TUNED=${3:?table} c5 > "$out/b_$i.json" 2> "$out/b_$i.err"
  echo "$i $(python3 -c "import json;print(json.load(open('$out/a_$i.json'))['value'], json.load(open('$out/b_$i.json'))['value'])")"
done

#!/bin/bash
# Alternating C3 (batch 8) bench lines: committed table vs another.   bash tools/ab/c3_ab.sh <tag> <pairs> <table>
set -e
out=gpurun_out/${1:?tag}
mkdir -p "$out"
for i in $(seq 1 "${2:?pairs}"); do
  timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/a_$i.json" 2> "$out/a_$i.err"
  DC_TUNED=${3:?table} timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline \
    > "$out/b_$i.json" 2> "$out/b_$i.err"
  echo "$i $(python3 -c "import json;print(json.load(open('$out/a_$i.json'))['value'], json.load(open('$out/b_$i.json'))['value'])")"
done

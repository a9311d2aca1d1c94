#!/bin/bash
# Resnet shortcut convs as a concurrent graph branch (unet.py _branch): DC_SIDE_STREAM=0 (one stream) against the
# default, alternating on one box -- C2 three pairs, C3 one pair -- then the GPU suite.
set -e
out=gpurun_out/r06p
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
for rep in 1 2 3; do
  DC_SIDE_STREAM=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_one_$rep.json" 2> "$out/c2_one_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_side_$rep.json" 2> "$out/c2_side_$rep.err"
  echo "c2 $rep $(v $out/c2_one_$rep.json) $(v $out/c2_side_$rep.json)"
done
DC_SIDE_STREAM=0 timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_one.json" 2> "$out/c3_one.err"
timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_side.json" 2> "$out/c3_side.err"
echo "c3 $(v $out/c3_one.json) $(v $out/c3_side.json)"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/gputest.log" 2>&1
tail -3 "$out/gputest.log"

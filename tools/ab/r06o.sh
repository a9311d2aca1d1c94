#!/bin/bash
# HIP runtime settings vs the per-launch floor and the C2 step: default, HIP_FORCE_DEV_KERNARG=1 (kernel
# arguments in device memory), DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (to learn whether packet capture is on by default).
set -e
out=gpurun_out/r06o
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
for e in "" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  env $e timeout -k 10 120 python -u tools/launch_floor_probe.py >> "$out/floor.jsonl"
done
cat "$out/floor.jsonl"
for rep in 1 2; do
  for e in "X=0" "HIP_FORCE_DEV_KERNARG=1"; do
    tag=${e%%=*}
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_${tag}_$rep.json" 2> "$out/c2_${tag}_$rep.err"
    echo "c2 $rep $e $(v $out/c2_${tag}_$rep.json)"
  done
done
echo done

#!/bin/bash
# Round 6: level-2/3 skinny launches with the weights cold (rotating copies past the Infinity Cache) against warm
# (one / two copies: Infinity-Cache resident) -- what a weight prefetch could buy at most.
set -e
out=gpurun_out/r06k
mkdir -p "$out"
export TMPDIR=/tmp
for s in l3 l2; do
  timeout -k 10 300 python -u tools/skinny_bench.py --set $s --tuned-only > "$out/${s}_cold.txt" 2>&1
  timeout -k 10 300 python -u tools/skinny_bench.py --set $s --tuned-only --copies 2 > "$out/${s}_warm2.txt" 2>&1
  timeout -k 10 300 python -u tools/skinny_bench.py --set $s --tuned-only --copies 1 > "$out/${s}_warm1.txt" 2>&1
done
echo done

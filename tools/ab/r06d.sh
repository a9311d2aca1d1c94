#!/bin/bash
# Round 6: attention block configurations per shape (DC_ATTN_CFG forced: forward ids 0-4, backward 0-2; SK off / forced)
set -e
out=gpurun_out/r06d
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/attn_bench.py --reps 3 > "$out/auto.txt" 2>&1
for c in 0 1 2 3 4; do
  DC_ATTN_CFG=$c timeout -k 10 200 python -u tools/attn_bench.py --reps 3 > "$out/cfg$c.txt" 2>&1
done
DC_ATTN_SK=2 timeout -k 10 200 python -u tools/attn_bench.py --reps 3 > "$out/sk2.txt" 2>&1
DC_ATTN_SK=0 timeout -k 10 200 python -u tools/attn_bench.py --reps 3 > "$out/sk0.txt" 2>&1
echo done

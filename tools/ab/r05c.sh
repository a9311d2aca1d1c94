#!/bin/bash
# round 5, box 2: attention before / after (ab/old = the tree before the forward's max / sum chains), the FF2 + proj_out
# fold probe, attention PMC passes
set -e
out=gpurun_out/r05c
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/attn_bench.py > "$out/attn_new.txt" 2>&1
(cd ab/old && timeout -k 10 300 python -u ../../tools/attn_bench.py) > "$out/attn_old.txt" 2>&1
timeout -k 10 300 python -u tools/attn_bench.py > "$out/attn_new2.txt" 2>&1
timeout -k 10 400 python -u tools/fuse_probe.py > "$out/fuse_probe.txt" 2>&1
bash tools/ab/pmc_attn.sh r05c

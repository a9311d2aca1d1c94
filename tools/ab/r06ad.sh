#!/bin/bash
# Attention block configurations per UNet level (tools/attn_bench.py under DC_ATTN_CFG=<i>; the default is the
# attn_cfg rule) -- does the rule pick the fastest forward / backward at every level?  (DC_ATTN_SK=0 also: the plain
# backward grid at level 0.)
set -e
out=gpurun_out/r06ad
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/attn_bench.py > "$out/cfg_default.txt" 2>&1
for c in 0 1 2 3 4; do
  DC_ATTN_CFG=$c timeout -k 10 200 python -u tools/attn_bench.py > "$out/cfg_$c.txt" 2>&1
done
DC_ATTN_SK=0 timeout -k 10 200 python -u tools/attn_bench.py > "$out/cfg_nosk.txt" 2>&1
for f in "$out"/cfg_*.txt; do echo "== $f"; grep -v amdgpu.ids "$f" | sed 's/(all.*//'; done

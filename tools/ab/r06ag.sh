#!/bin/bash
# The GroupNorm apply / backward-apply load-order variant adopted in-tree: the GPU suite and smoke on this tree, then
# C2 pairs against the previous norms.hip (ab/lib_nh.so).
set -e
out=gpurun_out/r06ag
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/gputest.log" 2>&1
tail -1 "$out/gputest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1
tail -1 "$out/smoke.txt"
for rep in 1 2 3; do
  DC_LIB=ab/lib_nh.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep old $(v $out/c2_old_$rep.json) new $(v $out/c2_new_$rep.json)"
done

#!/bin/bash
# The kept second-pass changes (guidance per-step kernels, upsample adjoint, clamp backward, single-launch GroupNorm
# forward vectors) against the committed sources of those files (ab/lib_oldx.so): C2 three pairs, C3 one; then this
# tree's C2 bench line with its CPU baseline and the smoke test.
set -e
out=gpurun_out/r06x
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
for rep in 1 2 3; do
  DC_LIB=ab/lib_oldx.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep old $(v $out/c2_old_$rep.json) new $(v $out/c2_new_$rep.json)"
done
DC_LIB=ab/lib_oldx.so timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_old.json" 2> "$out/c3_old.err"
timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_new.json" 2> "$out/c3_new.err"
echo "c3 old $(v $out/c3_old.json) new $(v $out/c3_new.json)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1
tail -2 "$out/smoke.txt"
timeout -k 10 600 python -u bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err"
echo "c2 line $(v $out/bench_c2.json)"

#!/bin/bash
# Load-issue order across the small kernels (GroupNorm apply / backward-apply / group, LayerNorm, guidance per-step
# kernels, skinny split-K reduce, upsample adjoint, clamp backward): the committed sources (ab/lib_oldall.so) and the
# tree with only the skinny reduce reverted (ab/lib_oldsk.so) against this tree, alternating on one box; then the GPU
# suite on this tree.
set -e
out=gpurun_out/r06v
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
for rep in 1 2 3; do
  DC_LIB=ab/lib_oldall.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep old $(v $out/c2_old_$rep.json) new $(v $out/c2_new_$rep.json)"
done
for rep in 1 2; do
  DC_LIB=ab/lib_oldsk.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_oldsk_$rep.json" 2> "$out/c2_oldsk_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new2_$rep.json" 2> "$out/c2_new2_$rep.err"
  echo "c2 $rep oldsk $(v $out/c2_oldsk_$rep.json) new $(v $out/c2_new2_$rep.json)"
done
DC_LIB=ab/lib_oldall.so timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_old.json" 2> "$out/c3_old.err"
timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_new.json" 2> "$out/c3_new.err"
echo "c3 old $(v $out/c3_old.json) new $(v $out/c3_new.json)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/gputest.log" 2>&1
tail -1 "$out/gputest.log"

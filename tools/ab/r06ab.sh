#!/bin/bash
# 8-wave cross-attention forward (C <= 384) with the output tables and residual rows issued with phase 1's loads,
# against the committed source (ab/lib_xh.so): launch times, kernel tests, C2 three pairs, C3 two pairs.
set -e
out=gpurun_out/r06ab
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
DC_LIB=ab/lib_xh.so timeout -k 10 120 python -u tools/cross_bench.py > "$out/cross_old.txt" 2>&1
timeout -k 10 120 python -u tools/cross_bench.py > "$out/cross_new.txt" 2>&1
paste "$out/cross_old.txt" "$out/cross_new.txt" | grep -v amdgpu.ids | grep fwd
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "cross" -x -q --timeout 120 --timeout-method thread > "$out/kt.log" 2>&1
tail -1 "$out/kt.log"
for rep in 1 2 3; do
  DC_LIB=ab/lib_xh.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep old $(v $out/c2_old_$rep.json) new $(v $out/c2_new_$rep.json)"
done
for rep in 1 2; do
  DC_LIB=ab/lib_xh.so timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_old_$rep.json" 2> "$out/c3_old_$rep.err"
  timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_new_$rep.json" 2> "$out/c3_new_$rep.err"
  echo "c3 $rep old $(v $out/c3_old_$rep.json) new $(v $out/c3_new_$rep.json)"
done

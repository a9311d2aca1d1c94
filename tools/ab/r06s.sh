#!/bin/bash
# LayerNorm kernels with every load issued up front (norms.hip) against the previous source (ab/lib_nold.so):
# launch times, the kernel tests, then C2 alternating pairs.
set -e
out=gpurun_out/r06s
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
DC_LIB=ab/lib_nold.so timeout -k 10 120 python -u tools/ln_bench.py > "$out/ln_old.txt" 2>&1
timeout -k 10 120 python -u tools/ln_bench.py > "$out/ln_new.txt" 2>&1
paste "$out/ln_old.txt" "$out/ln_new.txt" | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "layernorm or ln or cross" -x -q --timeout 120 --timeout-method thread > "$out/kt.log" 2>&1
tail -1 "$out/kt.log"
for rep in 1 2 3; do
  DC_LIB=ab/lib_nold.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep $(v $out/c2_old_$rep.json) $(v $out/c2_new_$rep.json)"
done

#!/bin/bash
# Cross-attention kernels with every global load issued up front (per-channel vectors / probabilities staged in LDS,
# unconditional clamped loads, the LN3 addend hoisted) against the previous crossattn.hip (ab/lib_xold.so): bitwise
# equality of the outputs, per-level launch times, the kernel tests, then C2 alternating pairs.
set -e
out=gpurun_out/r06r
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
DC_LIB=ab/lib_xold.so timeout -k 10 120 python -u tools/cross_bits.py "$out/bits_old.pt"
timeout -k 10 120 python -u tools/cross_bits.py "$out/bits_new.pt"
python tools/cross_bits.py --compare "$out/bits_old.pt" "$out/bits_new.pt" | tee "$out/bits.txt"
rm -f "$out"/bits_*.pt
DC_LIB=ab/lib_xold.so timeout -k 10 120 python -u tools/cross_bench.py > "$out/cross_old.txt" 2>&1
timeout -k 10 120 python -u tools/cross_bench.py > "$out/cross_new.txt" 2>&1
paste "$out/cross_old.txt" "$out/cross_new.txt" | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "cross" -x -q --timeout 120 --timeout-method thread > "$out/kt.log" 2>&1
tail -1 "$out/kt.log"
for rep in 1 2 3; do
  DC_LIB=ab/lib_xold.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep $(v $out/c2_old_$rep.json) $(v $out/c2_new_$rep.json)"
done

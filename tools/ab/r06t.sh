#!/bin/bash
# Attention kernels with the prologue row loads (Q / K, V / Q, dO, O, lse) issued together (attention.hip row8 /
# fix_row8) against the previous source (ab/lib_aold.so): bitwise equality, launch times, the kernel tests, C2 pairs.
set -e
out=gpurun_out/r06t
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
DC_LIB=ab/lib_aold.so timeout -k 10 120 python -u tools/attn_bits.py "$out/bits_old.pt"
timeout -k 10 120 python -u tools/attn_bits.py "$out/bits_new.pt"
python tools/attn_bits.py --compare "$out/bits_old.pt" "$out/bits_new.pt" | tee "$out/bits.txt"
rm -f "$out"/bits_*.pt
DC_LIB=ab/lib_aold.so timeout -k 10 200 python -u tools/attn_bench.py > "$out/attn_old.txt" 2>&1
timeout -k 10 200 python -u tools/attn_bench.py > "$out/attn_new.txt" 2>&1
paste "$out/attn_old.txt" "$out/attn_new.txt" | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > "$out/kt.log" 2>&1
tail -1 "$out/kt.log"
for rep in 1 2 3; do
  DC_LIB=ab/lib_aold.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep $(v $out/c2_old_$rep.json) $(v $out/c2_new_$rep.json)"
done

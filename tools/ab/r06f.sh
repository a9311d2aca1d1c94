#!/bin/bash
# Round 6: staggered key-split attention forward (this tree) vs the same code without the stagger (ab/lib_stag0.so)
# and the round-6 base (ab/lib_base.so): attention tests, microbenchmark, C2 alternating.
set -e
out=gpurun_out/r06f
mkdir -p "$out"
export TMPDIR=/tmp
for rep in 1 2; do
  DC_LIB=ab/lib_base.so timeout -k 10 200 python -u tools/attn_bench.py --reps 3 --no-bwd > "$out/base_$rep.txt" 2>&1
  DC_LIB=ab/lib_stag0.so timeout -k 10 200 python -u tools/attn_bench.py --reps 3 --no-bwd > "$out/stag0_$rep.txt" 2>&1
  timeout -k 10 200 python -u tools/attn_bench.py --reps 3 --no-bwd > "$out/stag1_$rep.txt" 2>&1
done
echo attn ok
for rep in 1 2 3; do
  for v in base stag0 tree; do
    if [ $v = tree ]; then
      timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_${v}_$rep.json" 2> "$out/c2_${v}_$rep.err"
    else
      DC_LIB=ab/lib_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_${v}_$rep.json" 2> "$out/c2_${v}_$rep.err"
    fi
    echo "$v $rep $(python -c "import json;d=json.load(open('$out/c2_${v}_$rep.json'));print(d['value'])")"
  done
done
echo done

#!/bin/bash
# Round 6: skinny weight loads nt (ab/lib_nt.so) and the fused GroupNorm-statistics epilogue's barriers without the
# workgroup fence (ab/lib_gnb.so) against this tree (ab/lib_base.so): their kernel tests, then C2 alternating.
set -e
out=gpurun_out/r06b
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "folded or skinny" --timeout 300 \
  --timeout-method thread > "$out/tests_base.log" 2>&1
DC_LIB=ab/lib_nt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "skinny" \
  --timeout 300 --timeout-method thread > "$out/tests_nt.log" 2>&1
DC_LIB=ab/lib_gnb.so timeout -k 10 600 python -u -m pytest tests/test_gpu_gn_fused.py tests/test_gpu_kernels.py -m gpu \
  -x -q -k "gn or skinny" --timeout 300 --timeout-method thread > "$out/tests_gnb.log" 2>&1
echo tests ok
for rep in 1 2 3; do
  for v in base nt gnb; do
    DC_LIB=ab/lib_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_${v}_$rep.json" 2> "$out/c2_${v}_$rep.err"
    echo "$v $rep $(python -c "import json;d=json.load(open('$out/c2_${v}_$rep.json'));print(d['value'])")"
  done
done
echo done

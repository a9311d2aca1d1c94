#!/bin/bash
# GroupNorm elementwise / single-launch kernels and the per-step guidance kernels (preview, latent norm / apply, sparse
# loss) with their loads issued up front, against the committed sources (ab/lib_gold.so: norms.hip, gn_acc.h and
# guidance.hip at HEAD): the GroupNorm and guidance tests, then C2 alternating pairs.
set -e
out=gpurun_out/r06u
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_gn_fused.py tests/test_gpu_guidance.py tests/test_gpu_kernels.py -k "gn or group or guid or preview or latent or sparse or loss" -x -q --timeout 300 --timeout-method thread > "$out/kt.log" 2>&1
tail -1 "$out/kt.log"
for rep in 1 2 3; do
  DC_LIB=ab/lib_gold.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep $(v $out/c2_old_$rep.json) $(v $out/c2_new_$rep.json)"
done
DC_LIB=ab/lib_gold.so timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_old.json" 2> "$out/c3_old.err"
timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > "$out/c3_new.json" 2> "$out/c3_new.err"
echo "c3 $(v $out/c3_old.json) $(v $out/c3_new.json)"

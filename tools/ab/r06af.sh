#!/bin/bash
# GroupNorm apply / backward-apply with the first row's loads raw and unconditional (clamped row) and the per-channel
# vectors (+ forward statistics) ahead of the fold, (ab/lib_nvar.so, the variant) against the committed norms.hip (the in-tree library): GroupNorm tests,
# in-step per-kernel times, C2 pairs.
set -e
out=gpurun_out/r06af
mkdir -p "$out"
export TMPDIR=/tmp
v() { python -c "import json;print(json.load(open('$1'))['value'])"; }
DC_LIB=ab/lib_nvar.so timeout -k 10 600 python -u -m pytest tests/test_gpu_gn_fused.py tests/test_gpu_kernels.py -k "gn or group" -x -q --timeout 300 --timeout-method thread > "$out/kt.log" 2>&1
tail -1 "$out/kt.log"
for arm in old new; do
  if [ $arm = new ]; then export DC_LIB=ab/lib_nvar.so; else unset DC_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/t_$arm" -o run --output-format csv -- \
    python3 tools/step_profile.py --out "$out/descs_$arm.json" > "$out/stepprof_$arm.log" 2>&1
  python3 tools/step_families.py "$out/t_$arm/run_kernel_trace.csv" 687 names > "$out/families_$arm.txt"
  rm -rf "$out/t_$arm"
done
unset DC_LIB
grep -h "gn_\|window" "$out/families_old.txt" "$out/families_new.txt"
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  DC_LIB=ab/lib_nvar.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_new_$rep.json" 2> "$out/c2_new_$rep.err"
  echo "c2 $rep old $(v $out/c2_old_$rep.json) new $(v $out/c2_new_$rep.json)"
done

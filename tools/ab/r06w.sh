#!/bin/bash
# (1) the cross-attention kernels at the tiny UNet widths (the chunk clamp fix); (2) per-family kernel time of the
# graph-replayed C2 step, committed sources (ab/lib_oldall.so) vs this tree; (3) the GPU suite.
set -e
out=gpurun_out/r06w
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "cross" -x -q --timeout 120 --timeout-method thread > "$out/kt.log" 2>&1
tail -1 "$out/kt.log"
for arm in old new; do
  if [ $arm = old ]; then export DC_LIB=ab/lib_oldall.so; else unset DC_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/t_$arm" -o run --output-format csv -- \
    python3 tools/step_profile.py --out "$out/descs_$arm.json" > "$out/stepprof_$arm.log" 2>&1
  python3 tools/step_families.py "$out/t_$arm/run_kernel_trace.csv" 687 names > "$out/families_$arm.txt"
  rm -rf "$out/t_$arm"
done
unset DC_LIB
paste "$out/families_old.txt" "$out/families_new.txt" | head -24
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/gputest.log" 2>&1
tail -1 "$out/gputest.log"

#!/bin/bash
# Round 6: attention backward row constants + both halves' S / dP first (ab/lib_a1.so), and the same with the ring's
# per-tile barrier as a raw s_barrier instead of __syncthreads (this tree, ab/lib_a2.so): kernel tests, then the
# attention microbenchmark and the C2 bench alternating the round-5 tree (ab/old) and these.
set -e
out=gpurun_out/r06a
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attention" --timeout 300 \
  --timeout-method thread > "$out/tests.log" 2>&1
echo tests ok
for rep in 1 2; do
  (cd ab/old && timeout -k 10 200 python -u tools/attn_bench.py --reps 3) > "$out/old_$rep.txt" 2>&1
  DC_LIB=ab/lib_a1.so timeout -k 10 200 python -u tools/attn_bench.py --reps 3 > "$out/a1_$rep.txt" 2>&1
  timeout -k 10 200 python -u tools/attn_bench.py --reps 3 > "$out/a2_$rep.txt" 2>&1
done
echo attn ok
for rep in 1 2; do
  (cd ab/old && timeout -k 10 300 python -u bench.py --no-cpu-baseline) > "$out/c2_old_$rep.json" 2> "$out/c2_old_$rep.err"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_a2_$rep.json" 2> "$out/c2_a2_$rep.err"
done
echo done

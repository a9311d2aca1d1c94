#!/bin/bash
# r02za: re-entry pass on HEAD -- full GPU suite, smoke, C2 bench (with the CPU baseline), kernel-trace stats of
# C2, per-shape conv breakdown of one C2 step, C3 batch-8 bench
set -e
out=gpurun_out/r02za
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gputest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/trace_bench.json 2> $out/trace.err
timeout -k 10 300 python -u tools/conv_breakdown.py > $out/conv_breakdown_c2.txt 2> $out/conv_breakdown.err
timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c3_b8.json 2> $out/bench_c3_b8.err
echo r02za done

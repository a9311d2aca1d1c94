#!/bin/bash
# r02l part 1: full GPU suite, smoke, C2 bench (with the CPU baseline), kernel-trace stats of C2
set -e
out=gpurun_out/r02l
mkdir -p $out
export TMPDIR=/tmp
[ -n "$SKIP_SUITE" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gputest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/trace_bench.json 2> $out/trace.err
echo r02l part 1 done

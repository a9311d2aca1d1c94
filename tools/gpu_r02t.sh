#!/bin/bash
# r02t: kernel-boundary floor (launch_bench), full GPU suite, smoke, C2 bench on the rebuilt tree
set -e
out=gpurun_out/r02t
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/launch_bench.bin 778 > $out/launch_bench.txt 2>&1
[ -n "$SKIP_SUITE" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gputest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err
echo r02t done

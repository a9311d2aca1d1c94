#!/bin/bash
# r02zk: full GPU suite, smoke and C2 bench on the final tree (GN first-row prefetch in)
set -e
out=gpurun_out/r02zk
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gputest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.err
echo r02zk done

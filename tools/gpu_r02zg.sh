#!/bin/bash
# r02zg: final check of the in-tree library (built from HEAD after the reverted experiments): smoke, kernel tests, C2 bench
set -e
out=gpurun_out/r02zg
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_session.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python -u bench.py > $out/bench_c2.json 2> $out/bench_c2.err
echo r02zg done

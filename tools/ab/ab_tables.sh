#!/bin/bash
# A/B of GEMM tables on the C2 bench (GPU box): bash tools/ab/ab_tables.sh tools/ab/a.json tools/ab/b.json ...
set -e
mkdir -p gpurun_out/ab
for t in "$@"; do
  name=$(basename $t .json)
  DC_TUNED=$t timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 4 > gpurun_out/ab/$name.json 2>/dev/null
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/ab/$name.json'));print(d['value'],d['roofline']['avg_launch_ms'])")"
done

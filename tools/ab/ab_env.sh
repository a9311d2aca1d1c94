#!/bin/bash
# A/B of environment settings on the C2 bench (GPU box), each line "name|ENV=.. ENV2=..":
#   bash tools/ab/ab_env.sh "base|" "korder|DC_KORDER=1" ...
set -e
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%|*}
  envs=${spec#*|}
  env $envs timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 4 > gpurun_out/ab/$name.json 2>/dev/null
  echo "$name [$envs] $(python -c "import json;d=json.load(open('gpurun_out/ab/$name.json'));print(d['value'],d['roofline']['avg_launch_ms'])")"
done

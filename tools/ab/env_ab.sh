#!/bin/bash
# A/B of environment settings on the C2 bench line, alternating on one box (REPS rounds, default 2):
#   bash tools/ab/env_ab.sh <tag> "" "DC_GN_GROUP=0" ...      ("" = the defaults)
set -e
tag=${1:?tag}; shift
out=gpurun_out/$tag
mkdir -p "$out"
for rep in $(seq 1 "${REPS:-2}"); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    # shellcheck disable=SC2086
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/v${i}_$rep.json" 2> "$out/v${i}_$rep.err"
    echo "[$e] $rep $(python -c "import json;print(json.load(open('$out/v${i}_$rep.json'))['value'])")"
  done
done

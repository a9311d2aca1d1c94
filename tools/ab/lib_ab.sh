#!/bin/bash
# A/B of two prebuilt libdcamd.so builds (DC_LIB) on a python script and the C2 bench (GPU box):
#   bash tools/ab/lib_ab.sh <tag> "<script args>" ab/lib_a.so ab/lib_b.so ...
set -e
tag=${1:?tag}; script=$2; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)_$rep
    if [ -n "$script" ]; then
      # shellcheck disable=SC2086
      DC_LIB=$lib timeout -k 10 200 python -u $script > "$out/$name.txt" 2> "$out/$name.err"
    fi
    DC_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 4 > "$out/$name.json" 2> "$out/$name.jerr"
    echo "$name $(python -c "import json;d=json.load(open('$out/$name.json'));print(d['value'])")"
  done
done

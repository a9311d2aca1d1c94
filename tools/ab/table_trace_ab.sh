#!/bin/bash
# A/B of GEMM tables on one box: a kernel trace of each table (bench.py --steps 2), then alternating C2 bench lines.
#   bash tools/ab/table_trace_ab.sh <tag> <pairs> <table A> <table B>   (a table "-" = the committed one)
set -e
out=gpurun_out/${1:?tag}
pairs=${2:?pairs}
ta=${3:?table A}
tb=${4:?table B}
mkdir -p "$out"
export TMPDIR=/tmp
arm() {   # arm <table> <command...>
  local t=$1
  shift
  if [ "$t" = "-" ]; then "$@"; else DC_TUNED=$t "$@"; fi
}
for x in a b; do
  t=$ta
  [ $x = b ] && t=$tb
  arm "$t" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace_$x" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$out/trace_$x.json" 2> "$out/trace_$x.err"
  echo "trace $x done"
done
for i in $(seq 1 "$pairs"); do
  for x in a b; do
    t=$ta
    [ $x = b ] && t=$tb
    arm "$t" timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/${x}_$i.json" 2> "$out/${x}_$i.err"
    echo "$x $i $(python3 -c "import json;print(json.load(open('$out/${x}_$i.json'))['value'])")"
  done
done

#!/bin/bash
# Re-tune the C3 / C4 / C5 shapes against the skinny variants (--try 43-47), keep only the swaps
# tools/ab/filter_table.py accepts, then alternate committed vs filtered table on C3, C4 and C5.
#   bash tools/ab/retune_c345.sh <tag>
set -e
out=gpurun_out/${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
DC_TUNE_COLD=2 timeout -k 10 900 python -u tools/tune_gemm.py --try 43 44 45 46 47 --workloads c2:8 c4:1 c5:1 \
  --out "$out/tuned_try.json" > "$out/tune.log" 2>&1
python3 tools/ab/filter_table.py depth_completion_amd/tuned_gfx950.json "$out/tuned_try.json" "$out/tuned_f.json" \
  > "$out/filter.log"
cat "$out/filter.log"
c3() { timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline; }
c4() { timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --no-cpu-baseline; }
c5() { timeout -k 10 400 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 --no-cpu-baseline; }
for w in c3 c4 c5; do
  for i in 1 2; do
    $w > "$out/${w}_a_$i.json" 2> "$out/${w}_a_$i.err"
    DC_TUNED=$out/tuned_f.json $w > "$out/${w}_b_$i.json" 2> "$out/${w}_b_$i.err"
    echo "$w $i $(python3 -c "import json;print(json.load(open('$out/${w}_a_$i.json'))['value'], json.load(open('$out/${w}_b_$i.json'))['value'])")"
  done
done

#!/bin/bash
# In-step variant choice for the C2 shapes (tools/ab/instep_tables.py): re-time every shape alone (top six kept), build
# three runner-up tables, profile the graph-replayed step under the committed table and each runner-up table, pick
# per shape.   bash tools/ab/instep_tune.sh <tag> [workload] [step_profile args] [top.json of an earlier run]
#   (with an earlier top.json: no re-tune, and the runner-ups after the first three are tried)
#   C2: c2:1   C3: c2:8 "--batch 8"   C4: c4:1 "--frame 352,1216,0,beams"   C5: c5:1 "--batch 10 --frame 900,1600,3000,uniform"
set -e
out=gpurun_out/${1:?tag}
wl=${2:-c2:1}
pargs=${3:-}
prev_top=${4:-}
mkdir -p "$out"
export TMPDIR=/tmp
T=depth_completion_amd/tuned_gfx950.json
if [ -n "$prev_top" ]; then
  cp "$prev_top" "$out/top.json"
  python3 tools/ab/instep_tables.py make $T "$out/top.json" "$out/alt" 3 3
else
  DC_TUNE_COLD=2 timeout -k 10 600 python -u tools/tune_gemm.py --fresh --workloads $wl --out "$out/fresh.json" \
    --top-out "$out/top.json" > "$out/tune.log" 2>&1
  echo "tune done"
  python3 tools/ab/instep_tables.py make $T "$out/top.json" "$out/alt" 3
fi
prof() {   # prof <name> <table>
  DC_TUNED=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/tr_$1" -o run --output-format csv -- \
    python3 tools/step_profile.py $pargs --out "$out/descs_$1.json" > "$out/prof_$1.log" 2>&1
  python3 tools/step_profile.py --trace "$out/tr_$1/run_kernel_trace.csv" --descs "$out/descs_$1.json" \
    --keys-out "$out/keys_$1.json" > "$out/shapes_$1.txt"
  head -2 "$out/shapes_$1.txt"
  rm -rf "$out/tr_$1"
}
prof c $T
for i in 1 2 3; do prof a$i "$out/alt$i.json"; done
python3 tools/ab/instep_tables.py pick $T "$out/instep.json" "$out/keys_c.json" \
  "$out/alt1.json" "$out/keys_a1.json" "$out/alt2.json" "$out/keys_a2.json" "$out/alt3.json" "$out/keys_a3.json" \
  | tee "$out/pick.log"

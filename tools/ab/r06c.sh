#!/bin/bash
# Round 6: the skinny two-kernel split-K shapes on one-launch alternatives, timed inside the graph-replayed C2 step
# (tools/ab/noreduce_tables.py): the committed table and three alternative tables profiled, per-shape pick.
set -e
out=gpurun_out/r06c
mkdir -p "$out"
export TMPDIR=/tmp
T=depth_completion_amd/tuned_gfx950.json
prof() {   # prof <name> <table>
  DC_TUNED=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/tr_$1" -o run --output-format csv -- \
    python3 tools/step_profile.py --out "$out/descs_$1.json" > "$out/prof_$1.log" 2>&1
  python3 tools/step_profile.py --trace "$out/tr_$1/run_kernel_trace.csv" --descs "$out/descs_$1.json" \
    --keys-out "$out/keys_$1.json" > "$out/shapes_$1.txt"
  head -2 "$out/shapes_$1.txt"
  rm -rf "$out/tr_$1"
}
prof c $T
for i in 1 2 3; do prof a$i tools/ab/nr_alt$i.json; done
python3 tools/ab/noreduce_tables.py pick $T "$out/noreduce.json" 0.03 "$out/keys_c.json" \
  tools/ab/nr_alt1.json "$out/keys_a1.json" tools/ab/nr_alt2.json "$out/keys_a2.json" tools/ab/nr_alt3.json \
  "$out/keys_a3.json" | tee "$out/pick.log"
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_c_$rep.json" 2> "$out/c2_c_$rep.err"
  DC_TUNED=$out/noreduce.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/c2_n_$rep.json" \
    2> "$out/c2_n_$rep.err"
  echo "$rep $(python -c "import json;print(json.load(open('$out/c2_c_$rep.json'))['value'], json.load(open('$out/c2_n_$rep.json'))['value'])")"
done
echo done

#!/bin/bash
# PMC counters per table key inside the graph-replayed C2 step, committed table vs another (tools/pmc_keys.py).
#   bash tools/ab/pmc_keys_ab.sh <tag> <table> <key substring>
set -e
out=gpurun_out/${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
for arm in a b; do
  n=0
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    n=$((n + 1))
    if [ $arm = a ]; then
      # shellcheck disable=SC2086
      timeout -s KILL 300 rocprofv3 --pmc $set -d "$out/${arm}_$n" -o run --output-format csv -- \
        python3 tools/step_profile.py --out "$out/descs_$arm.json" > "$out/${arm}_$n.log" 2>&1
    else
      # shellcheck disable=SC2086
      DC_TUNED=$2 timeout -s KILL 300 rocprofv3 --pmc $set -d "$out/${arm}_$n" -o run --output-format csv -- \
        python3 tools/step_profile.py --out "$out/descs_$arm.json" > "$out/${arm}_$n.log" 2>&1
    fi
    python3 tools/pmc_keys.py "$out/${arm}_$n/run_counter_collection.csv" "$out/descs_$arm.json" "$3" \
      > "$out/keys_${arm}_$n.txt"
    cat "$out/keys_${arm}_$n.txt"
    rm -rf "${out:?}/${arm}_$n"
  done
done

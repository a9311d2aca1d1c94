#!/bin/bash
# PMC passes over the attention kernels of tools/attn_bench.py (GPU box): issue / wait anatomy and LDS / MFMA
# counters, one counter set per run (rocprofv3 does not split counters over passes).  Counter names are checked
# against `rocprofv3 --list-avail` first; a set with an unknown name is skipped.
#   bash tools/ab/pmc_attn.sh <tag>
set -e
out=gpurun_out/${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$out/pmc_avail.txt" 2>&1 || true
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  n=$((n + 1))
  ok=1
  for c in $set; do
    grep -q "\b$c\b" "$out/pmc_avail.txt" || { echo "skip set $n: $c not listed" >> "$out/pmc_attn.log"; ok=0; }
  done
  [ $ok = 1 ] || continue
  # shellcheck disable=SC2086
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "attn_" -d "$out/pmc_attn_$n" -o run \
    --output-format csv -- python3 tools/attn_bench.py --reps 1 > "$out/pmc_attn_$n.txt" 2>&1
  echo "set $n done" >> "$out/pmc_attn.log"
done

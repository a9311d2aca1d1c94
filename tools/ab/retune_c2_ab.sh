#!/bin/bash
# Re-tune every C2 shape with DC_TUNE_COLD=<mode> (2: caches flushed, then the activation operands read back --
# the step's cache state, weights cold / inputs warm), then A/B the C2 bench line old vs new table, alternating.
# Usage: bash tools/ab/retune_c2_ab.sh <tag> <cold mode>
set -e
tag=${1:?tag}
mode=${2:-2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
DC_TUNE_COLD=$mode timeout -k 10 1200 python -u tools/tune_gemm.py --fresh --workloads c2:1 --out $out/tuned_c2.json \
  > $out/tune.log 2>&1
# merge: the C2 entries re-tuned, everything else from the committed table
python - <<PY
import json
old = {tuple(e["key"]): e for e in json.load(open("depth_completion_amd/tuned_gfx950.json"))}
new = {tuple(e["key"]): e for e in json.load(open("$out/tuned_c2.json"))}
old.update(new)
json.dump(list(old.values()), open("$out/tuned.json", "w"), indent=0)
print(len(new), "re-tuned of", len(old))
PY
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_old_$i.json 2> $out/c2_old_$i.err
  DC_TUNED=$out/tuned.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/c2_new_$i.json 2> $out/c2_new_$i.err
done
echo "retune $tag done"

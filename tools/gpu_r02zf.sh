#!/bin/bash
# r02zf: fresh cold-cache tuning of the C2 (batch 1) shapes on the current kernels (the committed entries predate the
# multiply-shift prologue), merged over the committed table; C2 bench A/B committed vs merged table
set -e
out=gpurun_out/r02zf
mkdir -p $out
export TMPDIR=/tmp
DC_TUNE_COLD=1 timeout -k 10 900 python -u tools/tune_gemm.py --fresh --workloads c2:1 --out $out/tuned_c2.json > $out/tune.log 2>&1
python - <<PY
import json
old = json.load(open("depth_completion_amd/tuned_gfx950.json"))
new = {tuple(e["key"]): e for e in json.load(open("$out/tuned_c2.json"))}
changed = 0
for e in old:
    k = tuple(e["key"])
    if k in new and (new[k]["algo"], new[k]["splitk"]) != (e["algo"], e["splitk"]):
        changed += 1
        e["algo"], e["splitk"] = new[k]["algo"], new[k]["splitk"]
json.dump(old, open("$out/tuned_merged.json", "w"), indent=0)
print("entries", len(old), "changed", changed, "c2 shapes", len(new))
PY
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_old_$i.json 2> $out/bench_old_$i.err
  DC_TUNED=$out/tuned_merged.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_new_$i.json 2> $out/bench_new_$i.err
done
echo r02zf done

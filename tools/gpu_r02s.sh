#!/bin/bash
# r02s: re-tune the C2 (batch 1) shapes with the step's cache state (caches flushed, activation operands read
# back: DC_TUNE_COLD=2), merge over the committed table, A/B the C2 bench
set -e
out=gpurun_out/r02s
mkdir -p $out
DC_TUNE_COLD=2 timeout -k 10 600 python -u tools/tune_gemm.py --fresh --workloads c2:1 --out $out/tuned_c2_warmA.json > $out/tune.log 2>&1
python -u - <<'PY'
import json
old = json.load(open("depth_completion_amd/tuned_gfx950.json"))
new = {tuple(e["key"]): e for e in json.load(open("gpurun_out/r02s/tuned_c2_warmA.json"))}
merged = [new.get(tuple(e["key"]), e) for e in old]
changed = sum(1 for e in old if tuple(e["key"]) in new and (new[tuple(e["key"])]["algo"], new[tuple(e["key"])]["splitk"]) != (e["algo"], e["splitk"]))
json.dump(merged, open("gpurun_out/r02s/tuned_merged.json", "w"), indent=0)
print("entries", len(merged), "re-tuned", len(new), "changed", changed)
PY
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_old_$i.json 2> $out/bench_old_$i.err
  DC_TUNED=gpurun_out/r02s/tuned_merged.json timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_new_$i.json 2> $out/bench_new_$i.err
done
echo r02s done

#!/bin/bash
# r02r: nearest-tuned-shape GEMM variants (dc_conv_pick, ABI 16): C4 with a C2/C3-only table, heuristic vs
# nearest shape, against the C4-tuned table; then the full GPU suite
set -e
out=gpurun_out/r02r
mkdir -p $out
c4="--height 352 --width 1216 --pattern beams --steps 4 --warmup 1 --no-cpu-baseline"
DC_TUNED=abtmp/tuned_c2c3.json DC_GEMM_NN=0 timeout -k 10 300 python -u bench.py $c4 > $out/c4_heuristic.json 2> $out/c4_heuristic.err
DC_TUNED=abtmp/tuned_c2c3.json timeout -k 10 300 python -u bench.py $c4 > $out/c4_nearest.json 2> $out/c4_nearest.err
timeout -k 10 300 python -u bench.py $c4 > $out/c4_tuned.json 2> $out/c4_tuned.err
DC_TUNED=abtmp/tuned_c2c3.json DC_GEMM_NN=0 timeout -k 10 300 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 1 --warmup 1 --no-cpu-baseline > $out/c5_heuristic.json 2> $out/c5_heuristic.err
DC_TUNED=abtmp/tuned_c2c3.json timeout -k 10 300 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 1 --warmup 1 --no-cpu-baseline > $out/c5_nearest.json 2> $out/c5_nearest.err
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gputest.log 2>&1
echo r02r done

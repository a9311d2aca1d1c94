mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v -s --timeout 250 --timeout-method thread -k baseline_config > gpurun_out/c45_t.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --height 352 --width 1216 --points 19000 --steps 3 --no-cpu-baseline > gpurun_out/bench_c4.json 2>/dev/null" \
 "timeout -k 10 200 python -u bench.py --height 900 --width 1600 --points 3000 --steps 3 --no-cpu-baseline > gpurun_out/bench_c5.json 2>/dev/null"

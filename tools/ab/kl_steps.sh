mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "timeout -k 10 300 python -u tools/ab/debug_kl.py > gpurun_out/dbg_kl.log 2>&1" \
 "timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -x -v --timeout 300 --timeout-method thread -k kl > gpurun_out/kl_m.log 2>&1" \
 "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 250 --timeout-method thread -k vae_original > gpurun_out/kl_p.log 2>&1"

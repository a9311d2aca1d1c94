#!/bin/bash
# r02o: the ill-conditioned closed-form + whole-map-loss pipeline tests across three builds: r02i (exact
# max tracking, separate delta pass), tau=0 (exact max tracking, delta in dQ), current (lazy rescale, delta in dQ)
set -e
out=gpurun_out/r02o
mkdir -p $out
for lib in base tau0; do
  DC_LIB=abtmp/libdcamd_$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -v -s --timeout 250 --timeout-method thread -k "closed_form_full_image or per_input_full or vae_original or full_unet" > $out/$lib.log 2>&1 || true
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -v -s --timeout 250 --timeout-method thread -k "closed_form_full_image or per_input_full or vae_original or full_unet" > $out/cur.log 2>&1 || true
echo r02o done

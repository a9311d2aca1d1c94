#!/bin/bash
# r02m: attention forward accuracy A/B (before / after the lazy-rescale + MFMA row-sum change), and the
# guided AutoencoderKL pipeline test that moved
set -e
out=gpurun_out/r02m
mkdir -p $out
DC_LIB=abtmp/libdcamd_base.so timeout -k 10 200 python -u tools/attn_acc.py > $out/acc_base.txt 2>&1
timeout -k 10 200 python -u tools/attn_acc.py > $out/acc_new.txt 2>&1
DC_LIB=abtmp/libdcamd_base.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -v -s --timeout 250 --timeout-method thread -k "vae_original" > $out/vae_base.log 2>&1 || true
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -v -s --timeout 250 --timeout-method thread -k "vae_original" > $out/vae_new.log 2>&1 || true
echo r02m done

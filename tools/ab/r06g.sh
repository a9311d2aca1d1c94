#!/bin/bash
set -e
out=gpurun_out/r06g
mkdir -p "$out"
export TMPDIR=/tmp
DC_LIB=ab/lib_stag0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k "attention_fwd" \
  --timeout 300 --timeout-method thread > "$out/tests_stag0.log" 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k "attention_fwd" --timeout 300 \
  --timeout-method thread > "$out/tests_stag1.log" 2>&1 || true
echo done

#!/bin/bash
set -e
out=gpurun_out/r06h
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/attn_repeat_probe.py > "$out/probe.txt" 2>&1
timeout -k 10 120 python -u tools/attn_repeat_probe.py --peak 1 > "$out/probe_p1.txt" 2>&1
timeout -k 10 120 python -u tools/attn_repeat_probe.py --t 6912 --peak 4 > "$out/probe_6912.txt" 2>&1
DC_LIB=ab/lib_stag0.so timeout -k 10 120 python -u tools/attn_repeat_probe.py > "$out/probe_stag0.txt" 2>&1
echo done

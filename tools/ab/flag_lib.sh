#!/bin/bash
# Link an A/B variant of libdcamd.so from the in-tree objects with some sources recompiled under extra flags (CPU):
#   bash tools/ab/flag_lib.sh <out.so> "<csrc files>" <extra flags...>
# e.g. bash tools/ab/flag_lib.sh ab/lib_nt.so "conv_skinny9.hip conv_skinny9_gn.hip" -DDC_SKINNY_WAUX=2
set -e
out=$1; files=$2; shift 2
tmp=$(mktemp -d)
trap 'rm -rf '"$tmp" EXIT
pids=()
for f in $files; do
  fl=(-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result)
  [ "$f" = attention.hip ] && fl+=(-fno-slp-vectorize)
  /opt/rocm/bin/hipcc "${fl[@]}" "$@" -c "depth_completion_amd/csrc/$f" -o "$tmp/$f.o" 2> "$tmp/$f.err" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
objs=()
for o in depth_completion_amd/build_obj/*.o; do
  b=$(basename "$o" .o)
  if [ -f "$tmp/$b.o" ]; then objs+=("$tmp/$b.o"); else objs+=("$o"); fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$out" "${objs[@]}"
echo "built $out"

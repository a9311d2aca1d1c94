#!/bin/bash
# Link an A/B variant of libdcamd.so from the in-tree objects with ONE source file recompiled from another path
# (CPU container):  bash tools/ab/variant_lib.sh <out.so> <csrc file name> <path of the variant source> [extra flags]
# e.g. bash tools/ab/variant_lib.sh ab/lib_a1.so attention.hip /tmp/attention_a1.hip
set -e
out=$1; name=$2; src=$3; shift 3
objs=()
tmp=$(mktemp -d)
cp "$src" depth_completion_amd/csrc/.variant_$name
trap 'rm -f depth_completion_amd/csrc/.variant_'"$name"'; rm -rf '"$tmp" EXIT
flags=(-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result)
[ "$name" = attention.hip ] && flags+=(-fno-slp-vectorize)
/opt/rocm/bin/hipcc "${flags[@]}" "$@" -x hip -c depth_completion_amd/csrc/.variant_$name -o "$tmp/v.o"
for o in depth_completion_amd/build_obj/*.o; do
  if [ "$(basename "$o")" = "$name.o" ]; then objs+=("$tmp/v.o"); else objs+=("$o"); fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$out" "${objs[@]}"
echo "built $out"

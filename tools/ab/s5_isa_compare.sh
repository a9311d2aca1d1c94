#!/bin/bash
# CPU-only look at the round-2 S = 5 ring abort (profiles/r02zc): rebuild the instantiation that aborted -- the
# conv_gemm.hip of commit 1831bf1 with the two ring entries that round 2 appended as algos 23 / 24 ({64,64,64,5},
# {64,64,64,3}) -- as device assembly, next to the current tree's id 37 ({64,64,64,5}), and compare the kernel
# descriptors (LDS segment, registers, scratch), the LDS-DMA destinations (M0), the LDS offsets of the epilogue
# staging, the vmcnt thresholds and the hand-off's memory operations.  No GPU.
# Usage: bash tools/ab/s5_isa_compare.sh [outdir]   (≈7 min of hipcc; existing r2.s / r4.s in outdir are reused)
set -euo pipefail
repo=$(cd "$(dirname "$0")/../.." && pwd)
out=${1:-/tmp/s5_isa}
mkdir -p "$out/r2"
git -C "$repo" archive 1831bf1 depth_completion_amd/csrc include | tar x -C "$out/r2"
python3 - "$out/r2/depth_completion_amd/csrc/conv_gemm.hip" <<'EOF'
import sys
p = sys.argv[1]
s = open(p).read()
s = s.replace("{64, 64, 32, 8}};", "{64, 64, 32, 8}, {64, 64, 64, 5}, {64, 64, 64, 3}};")
s = s.replace("DC_ALGO(22)\n", "DC_ALGO(22) DC_ALGO(23) DC_ALGO(24)\n")
open(p, "w").write(s)
EOF
flags=(-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result --cuda-device-only -S)
[ -s "$out/r2.s" ] || (cd "$out/r2/depth_completion_amd/csrc" && /opt/rocm/bin/hipcc "${flags[@]}" conv_gemm.hip -o "$out/r2.s")
[ -s "$out/r4.s" ] || (cd "$repo/depth_completion_amd/csrc" && /opt/rocm/bin/hipcc "${flags[@]}" conv_gemm.hip -o "$out/r4.s")
python3 - "$out/r2.s" "$out/r4.s" <<'EOF'
import collections, re, sys
def kernels(path, tag):
    s = open(path).read()
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
        name, body = m.group(1), m.group(2)
        if "conv_gemm_kernelILi64ELi64ELi64ELi5E" not in name:
            continue
        g = lambda k: re.search(r"\." + k + r" (\S+)", body).group(1)
        i = s.index(name + ": ;")
        code = s[i:s.index(".Lfunc_end", i)]
        ins = [l.strip() for l in code.split("\n")]
        ins = [l for l in ins if l and not l.startswith((".", ";")) and not l.endswith(":") and ": ;" not in l]
        ops = collections.Counter(l.split()[0] for l in ins)
        flags = re.search(r"ELi5E(.*?)EEv", name).group(1)
        print(f"{tag} S=5 {flags:16s} lds {g('amdhsa_group_segment_fixed_size')} scratch "
              f"{g('amdhsa_private_segment_fixed_size')} vgpr {g('amdhsa_next_free_vgpr')} sgpr "
              f"{g('amdhsa_next_free_sgpr')} instr {sum(ops.values())}")
        m0 = [l for l in ins if re.search(r"\bm0\b", l)]
        vm = dict(collections.Counter(re.findall(r"vmcnt[(]([0-9]+)[)]", code)))
        offs = [int(x) for x in re.findall(r"ds_\w+ .*offset:(\d+)", code)]
        m0set = sorted(set(re.sub(r"s[0-9]+", "sX", l) for l in m0))
        print(f"    M0 writes {len(m0)}: {m0set}")
        print(f"    LDS-DMA {sum(1 for l in ins if l.startswith('buffer_load') and ' lds' in l)}, "
              f"max ds offset {max(offs) if offs else None}, vmcnt {vm}")
        print(f"    hand-off: atomics {ops['global_atomic_add'] + ops['buffer_atomic_add']}, sc1 stores "
              f"{sum(1 for l in ins if l.startswith('buffer_store') and 'sc1' in l)}, sc1 loads "
              f"{sum(1 for l in ins if l.startswith('buffer_load') and 'sc1' in l)}, barriers {ops['s_barrier']}")
kernels(sys.argv[1], "1831bf1")
kernels(sys.argv[2], "current")
EOF

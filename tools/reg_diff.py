"""Per-kernel register / scratch / LDS comparison of two device-assembly builds (CPU).

A change whose effect depends on register allocation (epilogue preloads, extra epilogue state) cannot be A/B-ed by a
runtime switch inside one binary: both arms carry the same allocation.  Compare the builds instead:
    (cd depth_completion_amd/csrc && hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S conv_gemm.hip \\
        -o ../../gpurun_out/scratch/new.s)      # and the same for the old tree (git archive <rev> | tar x -C ...)
    python tools/reg_diff.py gpurun_out/scratch/old.s gpurun_out/scratch/new.s [--filter conv_gemm_kernel]
Prints every kernel whose VGPR count moved by more than 4 or whose scratch grew, with the waves per SIMD the unified
512-entry register file allows (granule 8) on each side.
"""
import argparse
import re


def kernels(path, filt):
    s = open(path).read()
    out = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
        name, body = m.group(1), m.group(2)
        if filt and filt not in name:
            continue
        g = lambda k: int(re.search(r"\." + k + r" (\S+)", body).group(1))  # noqa: E731
        out[name] = (g("amdhsa_next_free_vgpr"), g("amdhsa_private_segment_fixed_size"),
                     g("amdhsa_group_segment_fixed_size"))
    return out


def waves(vgpr):
    return min(8, 512 // max(8, (vgpr + 7) // 8 * 8))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("old")
    ap.add_argument("new")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    old, new = kernels(a.old, a.filter), kernels(a.new, a.filter)
    common = sorted(set(old) & set(new))
    moved = [k for k in common if abs(new[k][0] - old[k][0]) > 4 or new[k][1] > old[k][1]]
    print(f"{len(common)} kernels in both builds, {len(moved)} moved "
          f"({len(set(new) - set(old))} only in new, {len(set(old) - set(new))} only in old)")
    for k in moved:
        o, n = old[k], new[k]
        flag = "  <-- fewer waves" if waves(n[0]) < waves(o[0]) else ""
        print(f"{k[:96]}\n    vgpr {o[0]} -> {n[0]}  scratch {o[1]} -> {n[1]}  lds {o[2]} -> {n[2]}  "
              f"waves/SIMD {waves(o[0])} -> {waves(n[0])}{flag}")


if __name__ == "__main__":
    main()

"""Serialized global-load waits per kernel in a device-assembly file (CPU).

    (cd depth_completion_amd/csrc && hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S norms.hip \\
        -o ../../gpurun_out/scratch/norms.s)
    python tools/wait_scan.py gpurun_out/scratch/norms.s [--filter gn_]
Counts, per kernel, the vmcnt(0) waits that follow at least one global / buffer load issued since the previous such
wait (each one a memory round trip the wave cannot overlap), and prints the load (L) / full-wait (W) / store (S) /
barrier (B) / branch (|) sequence.  A lane-guarded load in a divergent branch that the compiler closes with a wait
shows up as a run of "LW".
"""
import argparse
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--filter", default="")
    ap.add_argument("--width", type=int, default=110)
    a = ap.parse_args()
    s = open(a.asm).read()
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S):
        name, body = m.group(1), m.group(2)
        if a.filter not in name:
            continue
        seq = []
        for line in body.split("\n"):
            t = line.strip()
            if re.match(r"(global|buffer)_load", t):
                seq.append("L")
            elif re.match(r"s_waitcnt.*vmcnt\(0\)", t):
                seq.append("W")
            elif re.match(r"(global|buffer)_store", t):
                seq.append("S")
            elif t.startswith("s_barrier"):
                seq.append("B")
            elif re.match(r"s_cbranch|s_branch", t):
                seq.append("|")
        rt, pend = 0, False
        for c in seq:
            if c == "L":
                pend = True
            elif c == "W" and pend:
                rt, pend = rt + 1, False
        print(f"{rt:3d} {''.join(seq)[:a.width]:{a.width}s} {name[:90]}")


if __name__ == "__main__":
    main()

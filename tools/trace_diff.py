"""Per-launch-configuration time of two rocprofv3 kernel traces (A/B of a table or a kernel change): the
(kernel template, grid) pairs whose total time moved, and the sum over a kernel-name filter.
Usage: python tools/trace_diff.py <trace A dir> <trace B dir> [name regex] [min ms]"""
import collections
import csv
import re
import sys


def load(d, pat):
    t, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if not re.search(pat, name):
            continue
        key = (re.sub(r"\(.*", "", name).removeprefix("void ")[:64], r["Grid_Size_X"])
        t[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        n[key] += 1
    return t, n


def main():
    a_dir, b_dir = sys.argv[1], sys.argv[2]
    pat = sys.argv[3] if len(sys.argv) > 3 else "."
    lim = float(sys.argv[4]) if len(sys.argv) > 4 else 0.5
    a, an = load(a_dir, pat)
    b, bn = load(b_dir, pat)
    print(f"{'A ms':>9} {'calls':>6} {'B ms':>9} {'calls':>6}  kernel, grid")
    for k in sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, 0) - a.get(k, 0))):
        if abs(b.get(k, 0) - a.get(k, 0)) > lim:
            print(f"{a.get(k, 0):9.2f} {an.get(k, 0):6d} {b.get(k, 0):9.2f} {bn.get(k, 0):6d}  {k[0]}, {k[1]}")
    print(f"total A {sum(a.values()):.2f} ms  B {sum(b.values()):.2f} ms")


if __name__ == "__main__":
    main()

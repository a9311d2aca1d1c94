"""Per-kernel breakdown of one pipeline call from a rocprofv3 kernel trace (CSV).

Finds the calls by their graph-replayed guided steps: the trace is split into calls at gaps longer
than --gap ms; the chosen call's kernels are grouped by (shortened) name.
Usage: python tools/trace_window.py run_kernel_trace.csv [--call -2] [--gap 5] [--steps 50]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--call", type=int, default=-2)
    ap.add_argument("--gap", type=float, default=5.0)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--min-kernels", type=int, default=2000)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    calls, cur = [], [rows[0]]
    for r in rows[1:]:
        if (r[0] - cur[-1][1]) / 1e6 > a.gap:
            calls.append(cur)
            cur = []
        cur.append(r)
    calls.append(cur)
    calls = [c for c in calls if len(c) >= a.min_kernels]
    c = calls[a.call]
    wall = (c[-1][1] - c[0][0]) / 1e6
    busy = sum(e - s for s, e, _ in c) / 1e6
    g = defaultdict(lambda: [0, 0.0])
    for s, e, n in c:
        k = short(n)
        g[k][0] += 1
        g[k][1] += (e - s) / 1e6
    print(f"{len(calls)} calls; call {a.call}: {len(c)} kernels, wall {wall:.2f} ms, kernel-busy {busy:.2f} ms, "
          f"per step {busy / a.steps:.3f} ms busy")
    for k, (n, ms) in sorted(g.items(), key=lambda kv: -kv[1][1]):
        print(f"{ms:9.3f} ms {100 * ms / busy:5.1f} %  x{n:6d}  {1e3 * ms / n:8.2f} us  {k}")


if __name__ == "__main__":
    main()

"""Itemise the per-call time outside the 50 graph-replayed guided steps (rocprofv3 kernel trace of bench.py).

Run on the GPU box:  rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python3 bench.py --steps 3 ...
then here:           python tools/call_timeline.py <dir>/run_kernel_trace.csv

A guided step ends with step_advance_kernel and a call starts its GPU work with preprocess_kernel.  For each pair of
consecutive calls the stretch from the end of call c's last guided step to the first kernel of call c+1's first
guided step holds call c's final decode, call c+1's setup kernels (encoder, guides, row sets), and the GPU idle time
the host leaves (synchronising reads, Python between launches).  Printed per stretch: GPU busy, GPU idle, the idle
gaps >= --gap us with the kernels around them, and busy time per kernel family.
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"[<(].*$", "", name)
    return name[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=20.0, help="list idle gaps at least this long (us)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    adv = [i for i, r in enumerate(rows) if "step_advance" in r[2]]
    pre = [i for i, r in enumerate(rows) if "preprocess_kernel" in r[2]]   # one per call (dc_preprocess_image)
    if len(pre) < 2:
        raise SystemExit("need at least two calls (preprocess_kernel) in the trace")
    walls = [(rows[adv[j]][1] - rows[adv[j - 1]][1]) / 1e6 for j in range(1, len(adv))
             if adv[j] - adv[j - 1] == adv[1] - adv[0]]
    med = statistics.median(walls)
    print(f"{len(rows)} kernels, {len(pre)} calls; median guided step wall {med:.3f} ms "
          f"({adv[1] - adv[0]} kernels per step)")
    for c in range(1, len(pre)):
        p = pre[c]
        last = max(i for i in adv if i < p)              # end of call c-1's last guided step
        first_adv = min(i for i in adv if i > p)         # call c's first guided step ...
        nxt = min(i for i in adv if i > first_adv)
        k = nxt - first_adv                              # ... has k kernels: it starts at first_adv - k + 1
        s0 = first_adv - k + 1
        t0, t1 = rows[last][1], rows[s0][0]
        seg = rows[last + 1:s0]
        busy = sum(e - s for s, e, _ in seg)
        print(f"\n--- from the end of call {c - 1}'s steps to call {c}'s first guided step: {(t1 - t0) / 1e6:.3f} ms "
              f"(GPU busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms), {len(seg)} kernels")
        fam = defaultdict(lambda: [0, 0])
        prev_end, prev_name = t0, "step_advance (call end)"
        for s, e, n in seg:
            g = s - prev_end
            if g >= a.gap * 1e3:
                print(f"  idle {g / 1e6:8.3f} ms  at +{(prev_end - t0) / 1e6:7.3f} ms  after {short(prev_name):40s} "
                      f"before {short(n)}")
            fam[short(n)][0] += 1
            fam[short(n)][1] += e - s
            prev_end, prev_name = max(prev_end, e), n
        g = t1 - prev_end
        if g >= a.gap * 1e3:
            print(f"  idle {g / 1e6:8.3f} ms  at +{(prev_end - t0) / 1e6:7.3f} ms  after {short(prev_name):40s} "
                  f"before the first guided step")
        for name, (cnt, ns) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
            print(f"    {ns / 1e6:8.3f} ms  x{cnt:4d}  {name}")


if __name__ == "__main__":
    main()

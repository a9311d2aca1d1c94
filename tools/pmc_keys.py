"""Per-table-key PMC counters of one graph-replayed step (CPU post-processing of a rocprofv3 --pmc run of
tools/step_profile.py): the step's conv dispatches (the last complete step between step_advance_kernel markers; a
two-kernel skinny split's reduce dispatch added to its conv) matched to the recorded launches by order, each counter
summed per conv_key.
Usage: python tools/pmc_keys.py <run_counter_collection.csv> <descs.json> [key substring ...]"""
import csv
import json
import sys
from collections import defaultdict

CONV = ("conv_gemm_kernel", "conv_halo_kernel", "conv_skinny_kernel", "conv_resident_kernel")


def main():
    rows = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(sys.argv[1])):
        d = int(r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    descs = json.load(open(sys.argv[2]))
    order = sorted(names)
    marks = [i for i, d in enumerate(order) if "step_advance_kernel" in names[d]]
    step = order[marks[-2] + 1:marks[-1]] if len(marks) >= 2 else order
    conv = []
    for d in step:
        if "skinny_reduce_kernel" in names[d] and conv:
            conv[-1][1].append(d)
        elif any(k in names[d] for k in CONV):
            conv.append((d, [d]))
    if len(conv) != len(descs):
        print(f"warning: {len(conv)} conv dispatches in the step, {len(descs)} launches recorded")
    per = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(int)
    for (d, ds), desc in zip(conv, descs):
        k = json.dumps(desc["key"])
        cnt[k] += 1
        for x in ds:
            for c, v in rows[x].items():
                per[k][c] += v
    want = sys.argv[3:]
    for k in sorted(per, key=lambda k: -sum(per[k].values())):
        if want and not any(w in k for w in want):
            continue
        vals = "  ".join(f"{c} {v / cnt[k]:.4g}" for c, v in sorted(per[k].items()))
        print(f"{k} x{cnt[k]}: per launch {vals}")


if __name__ == "__main__":
    main()

"""HBM bytes and MFMA busy of the dominant kernel family over ONE graph-replayed guided step (CPU post-processing).

The PMC passes run tools/step_profile.py (a C2 call whose guided steps are hipGraph replays, as bench.py times
them), one counter set per pass:
    rocprofv3 --pmc FETCH_SIZE -d <dir>/f -o run --output-format csv -- python3 tools/step_profile.py --out d.json
    rocprofv3 --pmc WRITE_SIZE ...   /   rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE ...
This script splits each pass's dispatch sequence at step_advance_kernel (one per guided step), takes the last
complete step, and sums the counters of the conv family there -- conv_gemm / conv_halo / conv_skinny (+ its
skinny_reduce) / conv_resident kernels, i.e. exactly the kernels that bench.py's measure_conv_kernel removes
when it drops the dc_conv_gemm launches from the step graph.  Bytes per step, and per dc_conv_gemm launch
(the reduce kernels' bytes charged to the launches they belong to, as in the timing).
Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE doubled (gfx950 wide-read undercount), WRITE_SIZE as is,
both KiB.
Usage: python tools/pmc_step.py <fetch.csv> <write.csv> <mfma.csv> <descs.json> <out.json>
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from depth_completion_amd.build import conv_family_hash  # noqa: E402

FAMILY = re.compile(r"conv_(gemm|halo|skinny|resident)_kernel|skinny_reduce")
LAUNCH = re.compile(r"conv_(gemm|halo|skinny|resident)_kernel")


def last_step(path, counters):
    """{counter: sum over the family's dispatches of the last complete step}, family dispatches, launches."""
    disp = {}
    vals = defaultdict(lambda: defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r["Dispatch_Id"])
            disp[d] = r["Kernel_Name"]
            if r["Counter_Name"] in counters:
                vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
    order = sorted(disp)
    marks = [i for i, d in enumerate(order) if "step_advance_kernel" in disp[d]]
    if len(marks) < 2:
        raise SystemExit(f"{path}: fewer than two step_advance_kernel dispatches")
    window = order[marks[-2] + 1:marks[-1] + 1]
    fam = [d for d in window if FAMILY.search(disp[d])]
    launches = sum(1 for d in fam if LAUNCH.search(disp[d]))
    tot = {c: sum(vals[d][c] for d in fam) for c in counters}
    return tot, len(fam), launches, len(window)


def main():
    fetch, write, mfma, descs, out = sys.argv[1:6]
    f, nf, lf, wf = last_step(fetch, ["FETCH_SIZE"])
    w, nw, lw, ww = last_step(write, ["WRITE_SIZE"])
    m, nm, lm, wm = last_step(mfma, ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"])
    with open(descs) as fh:
        n_calls = len(json.load(fh))
    fetch_b = 2.0 * 1024.0 * f["FETCH_SIZE"]
    write_b = 1024.0 * w["WRITE_SIZE"]
    res = {
        "population": "conv family of the last complete graph-replayed guided step (tools/step_profile.py)",
        # kernel sources + tuned table the counters were taken on; bench.py reports mfma_util only on a match
        "conv_family_hash": conv_family_hash(),
        "kernel_regex": FAMILY.pattern,
        "dc_conv_gemm_calls_per_step": n_calls,
        "family_dispatches_per_step": [nf, nw, nm],
        "launch_dispatches_per_step": [lf, lw, lm],
        "step_dispatches": [wf, ww, wm],
        "fetch_bytes_per_step": fetch_b,
        "write_bytes_per_step": write_b,
        "traffic_bytes_per_step": fetch_b + write_b,
        "traffic_bytes_per_launch": (fetch_b + write_b) / max(n_calls, 1),
        "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE as is; KiB -> bytes",
        "latent_shape": [1, 72, 96],
        "mfma_busy_cycles_per_step": m["SQ_VALU_MFMA_BUSY_CYCLES"],
        "grbm_gui_active_per_step": m["GRBM_GUI_ACTIVE"],
        # over the profiler's serialised dispatch windows (each dispatch's GRBM_GUI_ACTIVE includes its own ramp and
        # drain), so it reads below the graph-timed utilisation; bench.py normalises the busy cycles by the
        # graph-replayed family time instead (roofline.mfma_util)
        "mfma_util_pmc_window": (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
                                 if m["GRBM_GUI_ACTIVE"] else None),
        "mfma_util_pmc_window_def": "sum SQ_VALU_MFMA_BUSY_CYCLES / (sum GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) over the "
                                    "family's dispatches of the step, each dispatch serialised by the profiler",
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

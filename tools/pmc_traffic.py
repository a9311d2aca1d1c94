"""HBM traffic per dc_conv_gemm launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Correction per MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports half the bytes of a
wide (16 B / lane) streaming read -- global_load and buffer_load ... lds alike -- so it is doubled;
WRITE_SIZE is exact for 16-B stores.  rocprofv3's FETCH_SIZE / WRITE_SIZE are in KiB.
Usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv>
                                   <out.json> [--regex conv_gemm] [--latent-shape 1,72,96]
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def per_dispatch(path, counter, regex):
    vals, names = defaultdict(float), {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter or not re.search(regex, r["Kernel_Name"]):
                continue
            d = int(r["Dispatch_Id"])
            vals[d] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    return vals, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--regex", default="conv_gemm")
    ap.add_argument("--latent-shape", default="1,72,96", help="frames,h,w of the profiled step (C2 default)")
    ap.add_argument("--source", default="")
    ap.add_argument("--mfma", default=None, help="counter_collection.csv of the SQ_VALU_MFMA_BUSY_CYCLES / "
                                                 "GRBM_GUI_ACTIVE pass")
    a = ap.parse_args()
    fv, _ = per_dispatch(a.fetch, "FETCH_SIZE", a.regex)
    wv, _ = per_dispatch(a.write, "WRITE_SIZE", a.regex)
    nf, nw = len(fv), len(wv)
    fetch_b = 2.0 * 1024.0 * sum(fv.values()) / max(nf, 1)
    write_b = 1024.0 * sum(wv.values()) / max(nw, 1)
    res = {"kernel_regex": a.regex, "dispatches_fetch_pass": nf, "dispatches_write_pass": nw,
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "traffic_bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE as is; KiB -> bytes",
           "latent_shape": [int(v) for v in a.latent_shape.split(",")], "source": a.source}
    if a.mfma:
        # MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe busy cycles summed over the SIMDs; 16 per
        # v_mfma_f32_16x16x32_bf16) / (GRBM_GUI_ACTIVE / 8 XCDs = GPU cycles of the dispatch x 1024 SIMDs),
        # summed over every conv_gemm dispatch of the pass
        busy, _ = per_dispatch(a.mfma, "SQ_VALU_MFMA_BUSY_CYCLES", a.regex)
        gui, _ = per_dispatch(a.mfma, "GRBM_GUI_ACTIVE", a.regex)
        res["mfma_util"] = round(sum(busy.values()) / (sum(gui.values()) / 8.0 * 1024.0), 4)
        res["mfma_util_def"] = ("sum SQ_VALU_MFMA_BUSY_CYCLES / (sum GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) over the "
                                "conv_gemm dispatches of the pass")
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""Summarise tools/pmc_study.sh output: per config, per-dispatch averages of the counters and derived ratios.
Usage: python tools/pmc_study_summary.py gpurun_out/<tag>"""
import csv
import os
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            if "End_Timestamp" in r and r.get("Start_Timestamp"):
                dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    n = len(per)
    avg = defaultdict(float)
    for d in per.values():
        for k, v in d.items():
            avg[k] += v / n
    return avg, (sum(dur.values()) / len(dur) if dur else None), n


def main(root):
    for line in open(os.path.join(root, "index.txt")):
        tag, shape, algo, split = line.split()
        a, ta, na = load(os.path.join(root, f"{tag}_A", "run_counter_collection.csv"))
        b, tb, nb = load(os.path.join(root, f"{tag}_B", "run_counter_collection.csv"))
        wc = a["SQ_WAVE_CYCLES"]
        gpu_cyc = a["GRBM_GUI_ACTIVE"] / 8
        mf = a["SQ_INSTS_MFMA"]
        print(f"{tag} shape {shape} algo {algo} split {split}: {na} dispatches, kernel {ta:.1f} us (pass A), "
              f"gpu cycles {gpu_cyc:.0f} (clock {gpu_cyc / ta / 1e3 if ta else 0:.2f} GHz)")
        print(f"   wave-cycles: wait_any {a['SQ_WAIT_ANY'] / wc:.2f}  wait_inst_any {a['SQ_WAIT_INST_ANY'] / wc:.2f} "
              f"(lds {a['SQ_WAIT_INST_LDS'] / wc:.2f})  active_inst_any {a['SQ_ACTIVE_INST_ANY'] / wc:.2f}")
        print(f"   MFMA busy / (gpu cycles x 1024 SIMD) = {a['SQ_VALU_MFMA_BUSY_CYCLES'] / (gpu_cyc * 1024):.3f}; "
              f"mfma insts {mf:.0f}; per MFMA: valu {b['SQ_INSTS_VALU'] / mf:.2f} (incl. mfma) lds {b['SQ_INSTS_LDS'] / mf:.2f} "
              f"salu {b['SQ_INSTS_SALU'] / mf:.2f} vmem {b['SQ_INSTS_VMEM'] / mf:.2f}")
        print(f"   LDS: bank-conflict / idx-active {b['SQ_LDS_BANK_CONFLICT'] / max(b['SQ_LDS_IDX_ACTIVE'], 1):.3f}; "
              f"active_inst_lds {b['SQ_ACTIVE_INST_LDS'] / wc:.3f} active_inst_vmem {b['SQ_ACTIVE_INST_VMEM'] / wc:.3f} "
              f"(of wave cycles)")


if __name__ == "__main__":
    main(sys.argv[1])

"""The bench line's roofline bookkeeping (CPU): algorithmic FLOPs / bytes of a dc_conv_gemm launch (bench.conv_flops,
bench.conv_bytes) and the graph-step PMC post-processing (tools/pmc_step.py: the last complete step between
step_advance_kernel markers, the conv family's counters, the gfx950 FETCH_SIZE correction), on synthetic inputs."""
import csv
import json
import os
import subprocess
import sys
import types

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def desc(**kw):
    base = dict(nb=1, hin=72, win=96, cin=320, hout=72, wout=96, cout=320, kh=3, kw=3, mode=0, rows=None, nrows=0,
                resid=None)
    base.update(kw)
    return types.SimpleNamespace(**base)


def test_conv_flops_and_bytes():
    import bench
    d = desc()
    M, K = 72 * 96, 9 * 320
    assert bench.conv_flops(d) == 2.0 * M * 320 * K
    # activations in, weights, outputs -- each once, bf16
    assert bench.conv_bytes(d) == 2.0 * (M * 320 + 320 * K + M * 320)
    assert bench.conv_bytes(desc(resid=1)) == bench.conv_bytes(d) + 2.0 * M * 320
    # a stride-2 transposed gather counts a quarter of the taps
    assert bench.conv_flops(desc(mode=2)) == bench.conv_flops(d) / 4
    # a row-list launch counts its rows
    assert bench.conv_flops(desc(rows=1, nrows=100)) == 2.0 * 100 * 320 * K
    # a nearest-upsample input (mode 1) is read at its own, smaller size
    up = desc(mode=1, hin=36, win=48)
    assert bench.conv_bytes(up) == 2.0 * (36 * 48 * 320 + 320 * K + M * 320)


def _write_pmc(path, counters, per_step):
    """A counter-collection CSV of three guided steps: each step = markers + conv-family and other dispatches."""
    fields = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        did = 0
        for step in range(3):
            for name, vals in per_step(step):
                did += 1
                for c in counters:
                    w.writerow({"Dispatch_Id": did, "Kernel_Name": name, "Counter_Name": c, "Counter_Value": vals.get(c, 0)})
            did += 1
            for c in counters:
                w.writerow({"Dispatch_Id": did, "Kernel_Name": "step_advance_kernel(int*)", "Counter_Name": c,
                            "Counter_Value": 0})


def test_pmc_step_last_complete_step(tmp_path):
    def step(i):   # the counters grow with the step index: only the last complete one (i = 2) may be summed
        k = i + 1
        return [("void conv_gemm_kernel<64>(P)", {"FETCH_SIZE": 100 * k, "WRITE_SIZE": 10 * k,
                                                   "SQ_VALU_MFMA_BUSY_CYCLES": 1000 * k, "GRBM_GUI_ACTIVE": 800 * k}),
                ("void skinny_reduce_kernel<9>(P)", {"FETCH_SIZE": 5 * k, "WRITE_SIZE": 1 * k}),
                ("void conv_halo_kernel<8>(P)", {"FETCH_SIZE": 50 * k, "WRITE_SIZE": 5 * k,
                                                 "SQ_VALU_MFMA_BUSY_CYCLES": 500 * k, "GRBM_GUI_ACTIVE": 400 * k}),
                ("void attn_fwd_kernel<5>(P)", {"FETCH_SIZE": 999, "WRITE_SIZE": 999,
                                                "SQ_VALU_MFMA_BUSY_CYCLES": 999, "GRBM_GUI_ACTIVE": 999})]
    f, w_, m = tmp_path / "f.csv", tmp_path / "w.csv", tmp_path / "m.csv"
    _write_pmc(f, ["FETCH_SIZE"], step)
    _write_pmc(w_, ["WRITE_SIZE"], step)
    _write_pmc(m, ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"], step)
    descs = tmp_path / "d.json"
    descs.write_text(json.dumps([{}, {}]))   # two dc_conv_gemm calls per step
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_step.py"), str(f), str(w_), str(m), str(descs),
                    str(out)], check=True, capture_output=True)
    r = json.loads(out.read_text())
    # step 3 (k = 3): conv family only (the attention dispatch is excluded), FETCH_SIZE doubled, KiB -> bytes
    assert r["fetch_bytes_per_step"] == pytest.approx(2 * 1024 * (300 + 15 + 150))
    assert r["write_bytes_per_step"] == pytest.approx(1024 * (30 + 3 + 15))
    assert r["traffic_bytes_per_launch"] == pytest.approx((r["fetch_bytes_per_step"] + r["write_bytes_per_step"]) / 2)
    assert r["mfma_busy_cycles_per_step"] == pytest.approx(4500)
    assert r["family_dispatches_per_step"] == [3, 3, 3] and r["launch_dispatches_per_step"] == [2, 2, 2]

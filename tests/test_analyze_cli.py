"""analyze.py host surface: dataset / result pairing, batching, per-batch score means,
bin percentages and the results JSON files -- checked against the oracle's restatement of analyze.py
(oracle/analyze_ref.py) on CPU, with the batch sums supplied by a test-side stand-in for dc_depth_metrics
that follows the kernel's contract.  The kernel itself is checked on the GPU (tests/test_gpu_analyze.py)."""
import json
import math

import numpy as np
import pytest
import torch
from click.testing import CliRunner

from depth_completion_amd import io as dio
from depth_completion_amd.analyze import calc_bins, evaluate, main, scores_from_sums
from oracle import analyze_ref as A


def make_eval_tree(root, datasets=2, n=5, h=12, w=16, seed=0):
    """datasets with image/ + sparse/ PNGs and a result tree with dense/*.npy (one frame lacks its dense)."""
    from PIL import Image
    g = torch.Generator().manual_seed(seed)
    src, dst = root / "src", root / "dst"
    for k in range(datasets):
        img_dir, sp_dir = src / f"seq{k}" / "image", src / f"seq{k}" / "sparse"
        de_dir = dst / f"seq{k}" / "dense"
        for d in (img_dir, sp_dir, de_dir):
            d.mkdir(parents=True)
        for i in range(n):
            Image.fromarray(torch.randint(0, 256, (h, w, 3), generator=g, dtype=torch.uint8).numpy()).save(
                img_dir / f"{i:03d}.png")
            sp = torch.where(torch.rand(h, w, generator=g) < 0.3, 1 + 118 * torch.rand(h, w, generator=g),
                             torch.zeros(()))
            dio.encode_depth_png(sp, sp_dir / f"{i:03d}.png")
            if k == 1 and i == 2:
                continue  # no dense for this frame: skipped with a warning
            dense = (sp + 6 * torch.randn(h, w, generator=g)).clamp(min=-5) + 3
            if i % 2:
                np.save(de_dir / f"{i:03d}.npy", dense[None].numpy())
            else:
                np.savez(de_dir / f"{i:03d}.npz", dense[None].numpy())
    return src, dst


def kernel_contract(bins):
    """Test-side stand-in for dc_depth_metrics: (sum |e|, sum e^2, n) overall and per bin, in fp64."""
    def fn(de, sp, lo, hi):
        de, sp = de.reshape(-1).double(), sp.reshape(-1).double()
        m = sp.float() > 0
        s = sp.float().clamp(lo, hi)
        e = (de.float().clamp(lo, hi) - s)
        rows = [[e[m].abs().double().sum().item(), (e[m] * e[m]).double().sum().item(), float(m.sum())]]
        for b_lo, b_hi in bins:
            mb = m & (s >= b_lo) & (s <= b_hi)
            rows.append([e[mb].abs().double().sum().item(), (e[mb] * e[mb]).double().sum().item(), float(mb.sum())])
        return np.array(rows)
    return fn


def oracle_results(src, dst, bin_size=10.0, min_depth=0.0, max_depth=120.0, batch_size=2):
    """analyze.py:138-357 with the oracle's per-batch scores (oracle/analyze_ref.py)."""
    from depth_completion_amd.analyze import pair_paths
    bins = A.calc_bins(min_depth, max_depth, bin_size)
    per_ds = {}
    all_o = {m: [] for m in ("mae", "rmse")}
    all_b = [{m: [] for m in ("mae", "rmse")} for _ in bins]
    for ds in dio.find_dataset_dirs(src):
        sps, des = pair_paths(ds, dst / ds.relative_to(src))
        o = {m: [] for m in ("mae", "rmse")}
        for i in range(0, len(sps), batch_size):
            sp = dio.to_depth(torch.stack(dio.load_img_tensors(sps[i:i + batch_size])))
            de = torch.stack([torch.from_numpy(np.asarray(dio.load_array(p), dtype=np.float32))
                              for p in des[i:i + batch_size]])
            ov, _, bn = A.batch_scores(de, sp, ["mae", "rmse"], bins, min_depth, max_depth)
            for m in ov:
                o[m].append(ov[m])
                all_o[m].append(ov[m])
            for b, r in enumerate(bn):
                if r is not None:
                    for m in r[0]:
                        all_b[b][m].append(r[0][m])
        per_ds[ds.name] = {m: float(torch.stack(o[m]).mean()) for m in o}
    return per_ds, {m: float(torch.stack(all_o[m]).mean()) for m in all_o}, \
        [{m: float(torch.stack(b[m]).mean()) if b[m] else float("nan") for m in b} for b in all_b]


def test_calc_bins_and_scores():
    assert calc_bins(0.0, 120.0, 10.0) == A.calc_bins(0.0, 120.0, 10.0)
    assert calc_bins(2.5, 100.0, 7.5)[-1] == (92.5, 100.0)
    with pytest.raises(ValueError):
        calc_bins(5.0, 5.0, 1.0)
    s = scores_from_sums(np.array([6.0, 20.0, 4.0]), ["mae", "rmse"])
    assert s["mae"] == np.float32(1.5) and s["rmse"] == np.float32(math.sqrt(5.0))
    assert math.isnan(scores_from_sums(np.array([0.0, 0.0, 0.0]), ["mae"])["mae"])


def test_evaluate_matches_oracle(tmp_path):
    src, dst = make_eval_tree(tmp_path)
    bins = calc_bins(0.0, 120.0, 10.0)
    res = evaluate(src, dst, batch_size=2, metric_fn=kernel_contract(bins))
    per_ds, overall, binned = oracle_results(src, dst)
    for name, ref in per_ds.items():
        got = json.loads((dst / name / "results.json").read_text())
        for m in ref:
            assert got["overall"][m] == pytest.approx(ref[m], rel=1e-5)
        assert sum(b["percentage"] for b in got["binned"]) >= 99.9  # bins cover [0, 120] (edges counted twice)
    for m in overall:
        assert res["overall"][m] == pytest.approx(overall[m], rel=1e-5)
    for got_b, ref_b in zip(res["binned"], binned):
        for m in ref_b:
            if math.isnan(ref_b[m]):
                assert math.isnan(got_b["metrics"][m])
            else:
                assert got_b["metrics"][m] == pytest.approx(ref_b[m], rel=1e-5)
    assert json.loads((dst / "results_all.json").read_text())["overall"] == res["overall"]


def test_cli_arguments(tmp_path):
    src, dst = make_eval_tree(tmp_path, datasets=1, n=2)
    r = CliRunner().invoke(main, [str(src), str(dst), "--metrics", "psnr"])
    assert r.exit_code == 1   # no valid metrics (analyze.py:145-153)
    r = CliRunner().invoke(main, [str(tmp_path / "dst"), str(dst)])
    assert r.exit_code == 1   # no dataset directories

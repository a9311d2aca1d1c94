"""dc_depth_metrics (csrc/metrics.hip) and the analyze.py-compatible evaluation on the GPU, against the
oracle's restatement of analyze.py / utils.mae / utils.rmse (oracle/analyze_ref.py)."""
import math

import numpy as np
import pytest
import torch

from oracle import analyze_ref as A
from test_analyze_cli import kernel_contract, make_eval_tree, oracle_results

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("lo,hi,size,shape", [(0.0, 120.0, 10.0, (4, 1, 37, 53)), (2.5, 100.0, 3.5, (3, 1, 64, 80)),
                                              (1.0, 80.0, 100.0, (1, 1, 7, 9))])
def test_depth_metrics_kernel(lo, hi, size, shape):
    from depth_completion_amd.analyze import DepthMetrics, calc_bins, scores_from_sums
    g = torch.Generator().manual_seed(3)
    sp = torch.where(torch.rand(shape, generator=g) < 0.2, (torch.rand(shape, generator=g) * 255).round() * 120 / 255,
                     torch.zeros(()))
    sp.view(-1)[:20] = torch.tensor([10.0, 20.0, 30.0, 2.5, 100.0] * 4)   # exactly on bin edges
    de = sp + 10 * torch.randn(shape, generator=g) - 2
    bins = calc_bins(lo, hi, size)
    got = DepthMetrics("cuda:0", bins)(de, sp, lo, hi)
    ref = kernel_contract(bins)(de, sp, lo, hi)
    assert np.array_equal(got[:, 2], ref[:, 2])                     # point counts exact
    np.testing.assert_allclose(got[:, :2], ref[:, :2], rtol=1e-9, atol=1e-9)
    ov, n, bn = A.batch_scores(de, sp, ["mae", "rmse"], bins, lo, hi)
    s = scores_from_sums(got[0], ["mae", "rmse"])
    assert n == int(got[0, 2])
    for m in ov:
        assert s[m] == pytest.approx(float(ov[m]), rel=1e-5)
    for b, r in enumerate(bn):
        if r is None:
            assert got[1 + b, 2] == 0
            continue
        sb = scores_from_sums(got[1 + b], ["mae", "rmse"])
        for m in r[0]:
            assert sb[m] == pytest.approx(float(r[0][m]), rel=1e-5)


def test_evaluate_on_gpu(tmp_path):
    from depth_completion_amd.analyze import evaluate
    src, dst = make_eval_tree(tmp_path, datasets=2, n=5)
    res = evaluate(src, dst, batch_size=2)
    per_ds, overall, binned = oracle_results(src, dst)
    for m in overall:
        assert res["overall"][m] == pytest.approx(overall[m], rel=1e-5)
    for got_b, ref_b in zip(res["binned"], binned):
        for m in ref_b:
            assert (math.isnan(got_b["metrics"][m]) and math.isnan(ref_b[m])) or \
                got_b["metrics"][m] == pytest.approx(ref_b[m], rel=1e-5)

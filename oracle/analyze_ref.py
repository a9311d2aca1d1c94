"""CPU restatement of the reference's evaluation (TEST INFRASTRUCTURE ONLY -- never imported by the product).

Follows analyze.py:233-357 (per-batch overall / binned MAE and RMSE, per-dataset and all-dataset means,
bin percentages) with utils.calc_bins (utils.py:162-192), utils.mae / utils.rmse (utils.py:692-740) and
utils.to_depth (utils.py:1137-1158), in torch on the CPU, so tests can check the HIP path
(dc_depth_metrics + depth_completion_amd/analyze.py) against it.  Pinned by golden vectors made from the
reference's own functions (tests/golden/make_golden.py, unit_functions: calc_bins / mae / rmse).
"""
from __future__ import annotations

import torch


def calc_bins(lower_bound: float, upper_bound: float, bin_size: float) -> list[tuple[float, float]]:
    """utils.py:162-192."""
    if lower_bound >= upper_bound:
        raise ValueError(f"Lower bound {lower_bound} must be less than upper bound {upper_bound}")
    bins = []
    while lower_bound < upper_bound:
        bins.append((lower_bound, min(lower_bound + bin_size, upper_bound)))
        lower_bound += bin_size
    return bins


def mae(preds, targets, masks=None):
    """utils.py:692-714."""
    if masks is not None:
        preds = preds[masks]
        targets = targets[masks]
    return torch.mean(torch.abs(preds - targets))


def rmse(preds, targets, masks=None):
    """utils.py:717-740."""
    if masks is not None:
        preds = preds[masks]
        targets = targets[masks]
    return torch.sqrt(torch.mean((preds - targets) ** 2))


def batch_scores(denses, sparses, metrics, bin_ranges, min_depth, max_depth, calc_binned=True):
    """analyze.py:252-290 for one batch: (overall {metric: score}, n_pts, [per bin ({metric: score}, n) | None])."""
    mask = sparses > 0
    num_pts = int(mask.sum())
    sparses = sparses.clamp(min=min_depth, max=max_depth)
    denses = denses.clamp(min=min_depth, max=max_depth)
    overall = {m: (mae if m == "mae" else rmse)(denses, sparses, masks=mask) for m in metrics}
    binned = []
    if calc_binned:
        for lower, upper in bin_ranges:
            mb = mask & (sparses >= lower) & (sparses <= upper)
            if not torch.any(mb):
                binned.append(None)
                continue
            binned.append(({m: (mae if m == "mae" else rmse)(denses, sparses, masks=mb) for m in metrics},
                           int(mb.sum())))
    return overall, num_pts, binned

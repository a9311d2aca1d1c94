"""analyze.py-compatible evaluation of depth-completion results on MI355X.

    python -m depth_completion_amd.analyze DATASET_ROOT RESULT_ROOT [options]

Same arguments, defaults, per-dataset ``results.json`` and ``results_all.json`` as the reference
(analyze.py:20-357): for every dataset, each dense prediction (``RESULT_ROOT/<dataset>/dense/**.npy|npz``)
is paired with its 8-bit sparse LiDAR map (``DATASET_ROOT/<dataset>/sparse/**.png``); per batch the
MAE / RMSE over the LiDAR pixels (mask taken before clamping both maps to [min_depth, max_depth]),
overall and per depth bin, come from one ``dc_depth_metrics`` launch (csrc/metrics.hip); scores are the
mean of the per-batch scores, bin percentages the share of points.  There is no CPU path: ``--cuda``
is accepted for compatibility, the metrics always run on the GPU.
"""
from __future__ import annotations

import json
import logging
import math
import sys
from pathlib import Path

import click
import numpy as np
import torch

from . import _lib
from . import io as dio

logger = logging.getLogger("depth_completion_amd.analyze")
METRICS = ["mae", "rmse"]


def calc_bins(lower_bound: float, upper_bound: float, bin_size: float) -> list[tuple[float, float]]:
    """utils.py:162-192."""
    if lower_bound >= upper_bound:
        raise ValueError(f"Lower bound {lower_bound} must be less than upper bound {upper_bound}")
    bins = []
    while lower_bound < upper_bound:
        bins.append((lower_bound, min(lower_bound + bin_size, upper_bound)))
        lower_bound += bin_size
    return bins


class DepthMetrics:
    """dc_depth_metrics on one batch -> (sum |e|, sum e^2, count) overall and per bin (fp64)."""

    def __init__(self, device, bin_ranges):
        _lib.load()  # fail loudly without the HIP extension
        self.device = torch.device(device)
        self.nbins = len(bin_ranges)
        self.bins = torch.tensor(bin_ranges, dtype=torch.float32, device=self.device).reshape(-1).contiguous()
        ws = _lib.load().dc_depth_metrics_ws_bytes()
        self.ws = torch.empty(-(-ws // 8), dtype=torch.float64, device=self.device)
        self.res = torch.empty(1 + self.nbins, 3, dtype=torch.float64, device=self.device)

    def __call__(self, denses: torch.Tensor, sparses: torch.Tensor, min_depth: float, max_depth: float):
        d = denses.to(self.device, torch.float32).contiguous()
        s = sparses.to(self.device, torch.float32).contiguous()
        if d.numel() != s.numel():
            raise ValueError(f"dense {tuple(d.shape)} and sparse {tuple(s.shape)} sizes differ")
        _lib.call("dc_depth_metrics", d.data_ptr(), s.data_ptr(), d.numel(), float(min_depth), float(max_depth),
                  self.bins.data_ptr() if self.nbins else None, self.nbins, self.ws.data_ptr(),
                  self.res.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
        return self.res.cpu().numpy()


def scores_from_sums(sums: np.ndarray, metrics) -> dict:
    """utils.mae / utils.rmse (utils.py:692-740) from (sum |e|, sum e^2, n); an empty mask gives NaN like
    torch.mean of an empty tensor."""
    sa, ss, n = sums
    out = {}
    for m in metrics:
        if n == 0:
            out[m] = np.float32("nan")
        elif m == "mae":
            out[m] = np.float32(sa / n)
        else:
            out[m] = np.float32(math.sqrt(ss / n))
    return out


def pair_paths(dataset_dir: Path, result_dir: Path):
    """analyze.py:184-210: sparse PNGs (first of each stem) and their dense arrays."""
    sparse_dir = dataset_dir / dio.DATASET_DIR_NAME_SPARSE
    dense_dir = result_dir / dio.RESULT_DIR_NAME_DENSE
    sparse_paths, dense_paths, cache = [], [], set()
    for path in sorted(sparse_dir.rglob("*")):
        if path.suffix != ".png" or path.stem in cache:
            continue
        cache.add(path.stem)
        rel = path.relative_to(sparse_dir)
        dense_path = None   # utils.find_file_with_exts (utils.py:1189-1215)
        for cand in [dense_dir / rel] + [(dense_dir / rel).with_suffix(ext) for ext in dio.NPARRAY_EXTS]:
            if cand.is_file():
                dense_path = cand
                break
        if dense_path is None:
            logger.warning(f"No dense depth map found for {path} (skipped)")
            continue
        sparse_paths.append(path)
        dense_paths.append(dense_path)
    return sparse_paths, dense_paths


def _mean(xs) -> float:
    """torch.stack(scores).mean() in fp32; an empty bin gives NaN (the reference's torch.stack([]) raises)."""
    if len(xs) == 0:
        return float("nan")
    return float(np.mean(np.asarray(xs, dtype=np.float32), dtype=np.float32))


def evaluate(dataset_root: Path, result_root: Path, metrics=("mae", "rmse"), calc_binned_scores=True, bin_size=10.0,
             max_sparse_depth=120.0, max_depth=120.0, min_depth=0.0, batch_size=32, num_threads=8, device="cuda:0",
             metric_fn=None):
    """analyze.py:138-357.  Returns results_all (also written to RESULT_ROOT/results_all.json)."""
    metrics = [m for m in metrics if m in METRICS]
    if not metrics:
        raise ValueError("No valid metrics provided")
    dataset_dirs = dio.find_dataset_dirs(dataset_root)
    if not dataset_dirs:
        raise ValueError("No dataset directories found")
    bin_ranges = calc_bins(min_depth, max_depth, bin_size)
    fn = metric_fn or DepthMetrics(device, bin_ranges)
    all_overall = {m: [] for m in metrics}
    all_binned = [{m: [] for m in metrics} for _ in bin_ranges]
    all_pts, all_pts_binned = 0, [0] * len(bin_ranges)
    for dataset_dir in dataset_dirs:
        result_dir = result_root / dataset_dir.relative_to(dataset_root)
        if not result_dir.exists():
            logger.warning(f"No result directory found for {dataset_dir.name}. Skip this dataset")
            continue
        sparse_paths, dense_paths = pair_paths(dataset_dir, result_dir)
        if not sparse_paths:
            logger.warning(f"No dense & sparse depth map pairs found for {dataset_dir.name}. Skip this dataset")
            continue
        overall = {m: [] for m in metrics}
        binned = [{m: [] for m in metrics} for _ in bin_ranges]
        pts, pts_binned = 0, [0] * len(bin_ranges)
        for i in range(0, len(sparse_paths), batch_size):
            sp = dio.to_depth(torch.stack(dio.load_img_tensors(sparse_paths[i:i + batch_size], mode="RGB",
                                                               num_threads=num_threads)),
                              max_distance=max_sparse_depth)
            de = torch.stack([torch.from_numpy(np.asarray(dio.load_array(p), dtype=np.float32))
                              for p in dense_paths[i:i + batch_size]])
            sums = fn(de, sp, min_depth, max_depth)
            n = int(sums[0, 2])
            for m, v in scores_from_sums(sums[0], metrics).items():
                overall[m].append(v)
                all_overall[m].append(v)
            pts += n
            all_pts += n
            if calc_binned_scores:
                for b in range(len(bin_ranges)):
                    nb = int(sums[1 + b, 2])
                    if nb == 0:
                        continue
                    for m, v in scores_from_sums(sums[1 + b], metrics).items():
                        binned[b][m].append(v)
                        all_binned[b][m].append(v)
                    pts_binned[b] += nb
                    all_pts_binned[b] += nb
        results = {"overall": {m: _mean(overall[m]) for m in metrics}}
        logger.info(f"[{dataset_dir.name}]: " + ", ".join(f"{m}: {results['overall'][m]:.2f}" for m in metrics))
        if calc_binned_scores:
            results["binned"] = [
                {"range": (lo, hi), "metrics": {m: _mean(binned[b][m]) for m in metrics},
                 "percentage": (pts_binned[b] / pts) * 100 if pts else float("nan")}
                for b, (lo, hi) in enumerate(bin_ranges)]
        with (result_dir / "results.json").open("w") as f:
            json.dump(results, f, indent=2)
    results_all = {"overall": {m: _mean(all_overall[m]) for m in metrics}, "binned": []}
    if calc_binned_scores:
        results_all["binned"] = [
            {"range": (lo, hi), "metrics": {m: _mean(all_binned[b][m]) for m in metrics},
             "percentage": (all_pts_binned[b] / all_pts) * 100 if all_pts else float("nan")}
            for b, (lo, hi) in enumerate(bin_ranges)]
    with (result_root / "results_all.json").open("w") as f:
        json.dump(results_all, f, indent=2)
    return results_all


@click.command(help="Analyze results of depth completion.")
@click.argument("dataset_root", type=click.Path(exists=True, path_type=Path, file_okay=False, dir_okay=True))
@click.argument("result_root", type=click.Path(exists=True, path_type=Path, file_okay=False, dir_okay=True))
@click.option("--log", type=click.Path(path_type=Path), default=None)
@click.option("--log-level", type=click.Choice(["TRACE", "DEBUG", "INFO", "SUCCESS", "WARNING", "ERROR", "CRITICAL"]),
              default="INFO")
@click.option("--metrics", type=str, default="mae,rmse")
@click.option("--calc-binned-scores", type=bool, default=True)
@click.option("--bin-size", type=click.FloatRange(min=0, min_open=True), default=10.0)
@click.option("--max-sparse-depth", type=click.FloatRange(min=0, min_open=True), default=120.0)
@click.option("--max-depth", type=click.FloatRange(min=0, min_open=True), default=120.0)
@click.option("--min-depth", type=click.FloatRange(min=0), default=0.0)
@click.option("-bs", "--batch-size", type=click.IntRange(min=1), default=32)
@click.option("-nt", "--num-threads", type=click.IntRange(min=1), default=8)
@click.option("--cuda", type=bool, default=True)
def main(dataset_root, result_root, log, log_level, metrics, calc_binned_scores, bin_size, max_sparse_depth,
         max_depth, min_depth, batch_size, num_threads, cuda):
    level = {"TRACE": 5, "SUCCESS": 25}.get(log_level, getattr(logging, log_level, logging.INFO))
    logging.basicConfig(level=level, stream=sys.stderr, format="%(levelname)s %(message)s")
    if log is not None:
        log.parent.mkdir(parents=True, exist_ok=True)
        logging.getLogger().addHandler(logging.FileHandler(log))
    if not cuda:
        logger.warning("--cuda False: the metrics run on the GPU (dc_depth_metrics) regardless")
    ms = []
    for m in [x.strip() for x in metrics.split(",") if x.strip()]:
        if m not in METRICS:
            logger.error(f"Invalid metric: {m} (skipped)")
        else:
            ms.append(m)
    if not ms:
        logger.critical("No valid metrics provided")
        sys.exit(1)
    if not dio.find_dataset_dirs(dataset_root):
        logger.critical("No dataset directories found")
        sys.exit(1)
    evaluate(dataset_root, result_root, ms, calc_binned_scores, bin_size, max_sparse_depth, max_depth, min_depth,
             batch_size, num_threads)


if __name__ == "__main__":
    main()

"""predict.py-compatible CLI end to end on the GPU (tiny synthetic UNet, 2 frames)."""
import numpy as np
import pytest
import torch
from click.testing import CliRunner

from depth_completion_amd.predict import main
from tests.test_predict_cli import make_dataset

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("extra", [[], ["--train-latents", "False"], ["--vae", "original"],
                                   ["--loss-funcs", "l1,l2,edge", "--interp-mode", "nearest"]])
def test_cli_end_to_end(tmp_path, extra):
    make_dataset(tmp_path / "data", n=2, h=48, w=64)
    out = tmp_path / "out"
    r = CliRunner().invoke(main, [str(tmp_path / "data"), str(out), "--synthetic-weights", "0", "--unet-config",
                                  "tiny", "--res", "64", "--steps", "3", "--compress", "npy", "-vr", "64", "-1",
                                  *extra])
    assert r.exit_code == 0, (r.output, r.exception)
    dense = sorted((out / "dense" / "cam0").glob("*.npy"))
    vis = sorted((out / "vis" / "cam0").glob("*_vis.jpg"))
    assert [p.stem for p in dense] == ["0000", "0001"] and len(vis) == 2
    for p in dense:
        d = np.load(p)
        assert d.shape == (1, 48, 64) and np.isfinite(d).all() and d.min() >= 0.0 and d.max() <= 120.0


def test_cli_resume(tmp_path):
    """--resume re-runs only the frame whose output was removed; the others keep their files untouched."""
    make_dataset(tmp_path / "data", n=3, h=48, w=64)
    out = tmp_path / "out"
    args = [str(tmp_path / "data"), str(out), "--synthetic-weights", "0", "--unet-config", "tiny", "--res", "64",
            "--steps", "2", "--compress", "npy", "--vis", "False"]
    r = CliRunner().invoke(main, args)
    assert r.exit_code == 0, (r.output, r.exception)
    dense = sorted((out / "dense" / "cam0").glob("*.npy"))
    assert len(dense) == 3
    first = np.load(dense[1])
    mtimes = {p.name: p.stat().st_mtime_ns for p in dense}
    dense[1].unlink()
    r = CliRunner().invoke(main, args + ["--resume"])
    assert r.exit_code == 0, (r.output, r.exception)
    assert np.array_equal(np.load(dense[1]), first)          # the same frame, recomputed identically
    assert dense[0].stat().st_mtime_ns == mtimes[dense[0].name] and dense[2].stat().st_mtime_ns == mtimes[dense[2].name]


def test_cli_default_mode_matches_oracle(tmp_path, monkeypatch):
    """The dense maps the CLI writes in its default mode (guided per-step latents + learned affine, l1 + l2, TAESD,
    minmax) against the fp32 oracle run on the same frames, arguments and initial noise: the call's inputs and
    keyword arguments are recorded at the pipeline boundary, the oracle (same seeded synthetic weights as
    --synthetic-weights 0) replays them.  Bounds as the tiny-UNet pipeline tests: fitted |d| within 2x the bf16
    oracle's own error + 1e-3, and 2 % mean / 8 % p99 of the range."""
    from depth_completion_amd import pipeline as pl
    from depth_completion_amd.config import TINY
    from oracle.diffusers_ref import tiny_unet_config
    from tests.test_gpu_pipeline import ORACLE, build, fitted_error
    calls = []
    orig = pl.MarigoldDepthCompletionPipeline.__call__

    def spy(self, imgs, sparses, max_depth, **kw):
        d, lat = orig(self, imgs, sparses, max_depth, **kw)
        calls.append((imgs.cpu(), sparses.cpu(), max_depth, dict(kw), lat.shape))
        return d, lat

    monkeypatch.setattr(pl.MarigoldDepthCompletionPipeline, "__call__", spy)
    make_dataset(tmp_path / "data", n=2, h=48, w=64)
    out = tmp_path / "out"
    r = CliRunner().invoke(main, [str(tmp_path / "data"), str(out), "--synthetic-weights", "0", "--unet-config",
                                  "tiny", "--res", "64", "--steps", "3", "--compress", "npy", "--vis", "False"])
    assert r.exit_code == 0, (r.output, r.exception)
    assert len(calls) >= 1 and sum(c[0].shape[0] for c in calls) == 2   # the CLI's batches cover both frames
    dense = torch.stack([torch.from_numpy(np.load(p)) for p in sorted((out / "dense" / "cam0").glob("*.npy"))])
    assert dense.shape == (2, 1, 48, 64)
    oracles = {dt: build(tiny_unet_config(), TINY, dt, ORACLE)[0] for dt in (torch.float32, torch.bfloat16)}
    res = {torch.float32: [], torch.bfloat16: []}
    sps_all = []
    for imgs, sps, max_depth, kw, lshape in calls:
        assert kw.get("pred_latents_prev") is None   # (no --use-prev-latent: every call starts from its noise)
        # the pipeline's default initial noise: CPU torch.Generator(seed), [1, 4, h, w] bf16 (deviation 1)
        noise = torch.randn((1, 4, lshape[-2], lshape[-1]),
                            generator=torch.Generator().manual_seed(kw.get("seed", 2024)), dtype=torch.bfloat16)
        for dt, o in oracles.items():
            d, _ = o(imgs.to(ORACLE), sps.to(ORACLE), max_depth, init_noise=noise, **kw)
            res[dt].append(d.cpu())
        sps_all.append(sps)
    sps = torch.cat(sps_all)
    d32, d16 = torch.cat(res[torch.float32]), torch.cat(res[torch.bfloat16])
    mean_h, p99_h = fitted_error(dense, d32, sps)
    mean_b, p99_b = fitted_error(d16, d32, sps)
    print(f"\nCLI default mode (tiny UNet, 2 frames, 3 steps, {len(calls)} calls): written dense fitted |d| mean "
          f"{mean_h:.5f} p99 {p99_h:.5f} | oracle-bf16 mean {mean_b:.5f} p99 {p99_b:.5f}; call kwargs {sorted(calls[0][3])}")
    assert mean_h <= 2 * mean_b + 1e-3 and p99_h <= 2 * p99_b + 1e-3
    assert mean_h <= 0.02 and p99_h <= 0.08

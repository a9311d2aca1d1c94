"""predict.py-compatible CLI end to end on the GPU (tiny synthetic UNet, 2 frames)."""
import numpy as np
import pytest
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

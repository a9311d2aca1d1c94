"""predict.py host surface on CPU: dataset discovery, sparse PNG codec, writers,
visualisation helpers and the CLI's argument handling (dry run).  The GPU end-to-end run of the CLI
is in tests/test_gpu_predict.py."""
import numpy as np
import pytest
import torch
from click.testing import CliRunner

from depth_completion_amd import io as dio
from depth_completion_amd.predict import main


def make_dataset(root, n=3, h=24, w=32, seg=False):
    from PIL import Image
    img_dir, sp_dir = root / "image" / "cam0", root / "sparse" / "cam0"
    img_dir.mkdir(parents=True)
    sp_dir.mkdir(parents=True)
    g = torch.Generator().manual_seed(0)
    for i in range(n):
        img = torch.randint(0, 256, (h, w, 3), generator=g, dtype=torch.uint8).numpy()
        Image.fromarray(img).save(img_dir / f"{i:04d}.jpg")
        d = torch.where(torch.rand(h, w, generator=g) < 0.1, 5 + 100 * torch.rand(h, w, generator=g),
                        torch.zeros(()))
        dio.encode_depth_png(d, sp_dir / f"{i:04d}.png")
    if seg:
        (root / "segmask").mkdir()
        (root / "segmask" / "map.csv").write_text("id,name,r,g,b\n0,road,128,64,128\n1,car,0,0,142\n")
    (img_dir / "notes.txt").write_text("not an image")
    return root


def test_sparse_png_codec_roundtrip(tmp_path):
    d = torch.tensor([[0.0, 120.0], [60.0, 30.5]])
    dio.encode_depth_png(d, tmp_path / "s.png")
    t = dio.load_img_tensor(tmp_path / "s.png", "RGB")
    assert t.shape == (3, 2, 2) and t.dtype == torch.uint8
    depth = dio.to_depth(t[None])
    assert depth.shape == (1, 1, 2, 2)
    assert torch.allclose(depth[0, 0], (d * 255 / 120).round() * 120 / 255)


def test_dataset_discovery(tmp_path):
    make_dataset(tmp_path / "seqA")
    make_dataset(tmp_path / "nested" / "seqB", n=2)
    found = sorted(p.name for p in dio.find_dataset_dirs(tmp_path))
    assert found == ["seqA", "seqB"]
    assert dio.find_dataset_dirs(tmp_path / "seqA") == [tmp_path / "seqA"]
    imgs = dio.find_img_paths(tmp_path / "seqA" / "image")
    assert len(imgs) == 3 and all(p.suffix == ".jpg" for p in imgs)


@pytest.mark.parametrize("compress,ext", [("npy", ".npy"), ("npz", ".npz"), (None, ".npy")])
def test_save_tensor_formats(tmp_path, compress, ext):
    x = torch.rand(1, 5, 7, dtype=torch.float32).to(torch.bfloat16)
    p = tmp_path / f"d{ext}"
    dio.save_tensor(x, p, compress=compress)
    y = dio.load_array(p)
    assert y.dtype == np.float32 and np.array_equal(y, x.float().numpy())
    with pytest.raises(ValueError):
        dio.save_tensor(x, tmp_path / "bad.txt", compress=compress)


def test_visualize_and_grid(tmp_path):
    d = torch.linspace(0, 120, 64).view(1, 1, 8, 8)
    v = dio.visualize_depth(d, max_depth=120.0)
    assert v.shape == (1, 3, 8, 8) and v.dtype == torch.uint8
    assert tuple(v[0, :, 0, 0].tolist()) == (158, 1, 66) and tuple(v[0, :, -1, -1].tolist()) == (94, 79, 162)
    with pytest.raises(ValueError):
        dio.visualize_depth(d, max_depth=0.0, min_depth=1.0)
    g = dio.make_grid([v[0], v[0], v[0]])
    assert g.shape == (3, 8 + 4, 3 * (8 + 2) + 2) and g[:, :2].sum() == 0
    r = dio.make_grid([v[0], v[0]], resize=(40, -1))
    assert r.shape[1] == 40 and r.dtype == torch.uint8
    dio.save_img_tensor(r, tmp_path / "v.jpg")
    assert (tmp_path / "v.jpg").stat().st_size > 0


def test_segmap_and_segmask(tmp_path):
    make_dataset(tmp_path / "s", seg=True)
    m = dio.load_segmap(tmp_path / "s" / "segmask" / "map.csv")
    assert m["name"] == ["road", "car"] and m["color"][1] == (0, 0, 142)
    img = torch.zeros(1, 3, 2, 2, dtype=torch.uint8)
    img[0, :, 1, 1] = torch.tensor([0, 0, 142])
    assert dio.to_segmask(img, m["color"])[0, 0].tolist() == [[0, 0], [0, 1]]


def test_cli_dry_run_and_coercions(tmp_path):
    make_dataset(tmp_path / "data")
    r = CliRunner().invoke(main, [str(tmp_path / "data"), str(tmp_path / "out"), "--dry-run",
                                  "--loss-funcs", "l1,bogus,l2", "-vo", "image,dense"])
    assert r.exit_code == 0, r.output
    lines = [ln for ln in r.output.splitlines() if ln.startswith("data\t")]
    assert len(lines) == 3 and all(ln.endswith(".png") for ln in lines)
    r = CliRunner().invoke(main, [str(tmp_path / "data"), str(tmp_path / "out"), "--model", "lcm"])
    assert r.exit_code != 0
    r = CliRunner().invoke(main, [str(tmp_path / "data"), str(tmp_path / "out")])  # no weights given
    assert r.exit_code != 0
    r = CliRunner().invoke(main, [str(tmp_path), str(tmp_path / "out2"), "--dry-run", "--steps", "0"])
    assert r.exit_code != 0  # IntRange(min=1)


def test_resume_pending_pairs(tmp_path):
    """--resume drops the pairs whose every output exists; a pair with one output missing is re-run."""
    from depth_completion_amd.predict import discover, frame_outputs, pending_pairs
    root = make_dataset(tmp_path / "data", n=3)
    (d, pairs, _), = discover(root, False)
    img_dir, sp_dir, out = d / "image", d / "sparse", tmp_path / "out"
    assert pending_pairs(pairs, out, img_dir, sp_dir, "npy", True, True) == pairs
    done = frame_outputs(out, img_dir, sp_dir, *pairs[0][:2], "npy", True, True)
    half = frame_outputs(out, img_dir, sp_dir, *pairs[1][:2], "npy", True, True)
    assert done[0].name == "0000.npy" and done[1].name == "0000_vis.jpg"
    for p in done + half[:1]:
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(b"x")
    assert pending_pairs(pairs, out, img_dir, sp_dir, "npy", True, True) == pairs[1:]
    assert pending_pairs(pairs, out, img_dir, sp_dir, "npy", True, False) == pairs[2:]   # vis off: dense suffices
    assert pending_pairs(pairs, out, img_dir, sp_dir, "npz", True, False) == pairs        # other format: pending

"""Dataset and result IO of the predict.py host surface.

Mirrors the reference's utils.py helpers used by predict.py:
* dataset layout ``<dataset>/image/...`` + ``<dataset>/sparse/...png`` (+ optional ``segmask/``),
  discovered recursively (utils.py:193-227, 1161-1187);
* 8-bit sparse depth PNG codec: depth = max_distance * R / 255 (utils.py:1137-1158);
* dense writers ``.npy`` / ``.npz`` (utils.py:592-689; ``.bl2`` needs blosc2, absent in this image);
* visualisation: Spectral colour map (utils.py:370-432), torchvision-style grid + bilinear resize
  (utils.py:973-1066), image save with torchvision's float->uint8 rounding (utils.py:533-589).
Images are decoded with PIL (the reference uses OpenCV, absent here); both give 8-bit RGB.
Colour-map and grid outputs are "parity unpinned" (no reference fixture covers them).
"""
from __future__ import annotations

import concurrent.futures
import csv
import os
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

DATASET_DIR_NAME_SPARSE = "sparse"     # utils.py:20-24
DATASET_DIR_NAME_IMAGE = "image"
DATASET_DIR_NAME_SEGMASK = "segmask"
RESULT_DIR_NAME_DENSE = "dense"
RESULT_DIR_NAME_VIS = "vis"
NPARRAY_EXTS = [".npy", ".npz", ".bl2"]

# ColorBrewer "Spectral" anchors (matplotlib's Spectral LinearSegmentedColormap, 11 colours)
_SPECTRAL = np.array([[158, 1, 66], [213, 62, 79], [244, 109, 67], [253, 174, 97], [254, 224, 139],
                      [255, 255, 191], [230, 245, 152], [171, 221, 164], [102, 194, 165], [50, 136, 189],
                      [94, 79, 162]], dtype=np.float64) / 255.0


def is_dataset_dir(path: Path) -> bool:
    return path.is_dir() and (path / DATASET_DIR_NAME_SPARSE).is_dir() and (path / DATASET_DIR_NAME_IMAGE).is_dir()


def find_dataset_dirs(root: Path) -> list[Path]:
    """utils.py:210-227: the root itself, else every nested dataset directory."""
    root = Path(root)
    if is_dataset_dir(root):
        return [root]
    return [p for p in root.rglob("*") if is_dataset_dir(p)]


def is_img_file(path: Path) -> bool:
    if not path.is_file():
        return False
    try:
        from PIL import Image
        with Image.open(path) as im:
            im.verify()
        return True
    except Exception:
        return False


def find_img_paths(root: Path) -> list[Path]:
    return [p for p in Path(root).rglob("*") if is_img_file(p)]


def load_img_tensor(path: Path, mode: str | None = "RGB") -> torch.Tensor | None:
    """[C, H, W] uint8, or None if unreadable (utils.py:817-857)."""
    from PIL import Image
    try:
        with Image.open(path) as im:
            if mode is not None:
                im = im.convert(mode)
            arr = np.asarray(im).copy()
    except Exception:
        return None
    if arr.size == 0:
        return None
    t = torch.from_numpy(arr)
    return t.unsqueeze(0) if t.ndim == 2 else t.permute(2, 0, 1).contiguous()


def load_img_tensors(paths: list[Path], mode: str | None = "RGB", num_threads: int = 1):
    if not paths:
        return []
    if num_threads <= 1:
        return [load_img_tensor(p, mode) for p in paths]
    with concurrent.futures.ThreadPoolExecutor(max_workers=num_threads) as ex:
        return list(ex.map(lambda p: load_img_tensor(p, mode), paths))


def to_depth(imgs: torch.Tensor, dtype=torch.float32, max_distance: float = 120.0) -> torch.Tensor:
    """utils.py:1137-1158: [N, 3, H, W] 8-bit range image -> [N, 1, H, W] metres from channel 0."""
    return max_distance * (imgs.to(dtype)[:, 0] / 255.0).unsqueeze(1)


def encode_depth_png(depth: torch.Tensor, path: Path, max_distance: float = 120.0) -> None:
    """Inverse of to_depth (the 8-bit sparse format predict.py consumes): R=G=B=round(255 d / max)."""
    from PIL import Image
    k = (depth.float().squeeze().clamp(0, max_distance) * 255.0 / max_distance).round().to(torch.uint8).numpy()
    Image.fromarray(np.stack([k, k, k], -1)).save(path)


def load_segmap(csv_path: Path) -> dict:
    """utils.py:230-323: map.csv with columns id, name, r, g, b -> names / RGB colours indexed by id."""
    with open(csv_path, newline="") as f:
        data = list(csv.reader(f))
    header, rows = data[0], [r for r in data[1:] if r and any(c.strip() for c in r)]
    missing = [c for c in ("id", "name", "r", "g", "b") if c not in header]
    if missing:
        raise ValueError(f"Missing required columns in CSV file: {', '.join(missing)}")
    col = {c: header.index(c) for c in ("id", "name", "r", "g", "b")}
    recs = [(int(r[col["id"]]), r[col["name"]], tuple(int(r[col[c]]) for c in "rgb")) for r in rows]
    n = max(i for i, _, _ in recs) + 1 if recs else 0
    ret = {"name": [""] * n, "color": [(0, 0, 0)] * n}
    for i, name, rgb in recs:
        ret["name"][i] = name
        ret["color"][i] = rgb
    return ret


def to_segmask(imgs: torch.Tensor, colormap) -> torch.Tensor:
    """utils.py:1084-1134: RGB class colours -> class ids [N, 1, H, W]."""
    if imgs.ndim != 4 or imgs.shape[1] != 3:
        raise ValueError("Input must be a 4D tensor with shape [N, 3, H, W]")
    n, _, h, w = imgs.shape
    out = torch.zeros(n, 1, h, w, dtype=imgs.dtype, device=imgs.device)
    for cid, rgb in enumerate(colormap):
        m = (imgs == torch.tensor(rgb, dtype=imgs.dtype, device=imgs.device).view(1, 3, 1, 1)).all(1, keepdim=True)
        out[m] = cid
    return out


def has_nan(x) -> bool:
    return bool(torch.isnan(x).any().item()) if isinstance(x, torch.Tensor) else bool(np.isnan(x).any())


def filterout(li: list, flags: list[bool]) -> list:
    if len(li) != len(flags):
        raise ValueError(f"Length of list {len(li)} must be equal to length of flags {len(flags)}")
    return [x for x, f in zip(li, flags) if f]


def _atomic_path(path: Path) -> Path:
    """Temporary sibling of ``path`` (same directory and suffix): writers fill it, then os.replace() moves it into
    place, so an existing output file is always a complete one (predict.py --resume skips existing outputs)."""
    return path.with_name(f".{path.stem}.{os.getpid()}.tmp{path.suffix}")


def save_tensor(x: torch.Tensor, path: Path, compress: str | None = None) -> None:
    """utils.py:592-689 (.npy / .npz; .bl2 needs blosc2).  Written atomically (temporary file + rename)."""
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    if torch.is_floating_point(x) and x.dtype not in (torch.float32, torch.float64):
        x = x.to(torch.float32)
    arr = x.detach().cpu().numpy()
    want = {None: ".npy", "npy": ".npy", "npz": ".npz", "bl2": ".bl2"}[compress]
    if path.suffix != want:
        raise ValueError(f"Invalid extension: {path.suffix} (must be {want})")
    tmp = _atomic_path(path)
    try:
        if compress == "bl2":
            try:
                import blosc2
            except ImportError as e:
                raise RuntimeError("compress=bl2 needs the blosc2 package, which is not installed") from e
            blosc2.save_array(arr, str(tmp), mode="w")
        else:
            with open(tmp, "wb") as f:
                if compress == "npz":
                    np.savez_compressed(f, arr)
                else:
                    np.save(f, arr)
        os.replace(tmp, path)
    finally:
        if tmp.exists():
            tmp.unlink()


def load_array(path: Path) -> np.ndarray:
    path = Path(path)
    if path.suffix not in NPARRAY_EXTS:
        raise ValueError(f"Invalid extension: {path.suffix} (must be one of {NPARRAY_EXTS}")
    if path.suffix == ".npz":
        return np.load(path)["arr_0"]
    if path.suffix == ".bl2":
        import blosc2
        return blosc2.load_array(str(path))
    return np.load(path)


def colormap_spectral(x: torch.Tensor) -> torch.Tensor:
    """[H, W] in [0, 1] -> [H, W, 3] uint8, matplotlib Spectral (256-entry LUT, nearest lookup)."""
    lut = np.stack([np.interp(np.linspace(0, 1, 256), np.linspace(0, 1, 11), _SPECTRAL[:, c]) for c in range(3)], -1)
    lut = torch.from_numpy((lut * 255.0).round().astype(np.uint8))
    idx = (x.float().clamp(0, 1) * 255.0).to(torch.long).cpu()
    return lut[idx]


def visualize_depth(depth_maps: torch.Tensor, max_depth: float, min_depth: float = 0.0) -> torch.Tensor:
    """utils.py:370-432: [N, 1, H, W] metres -> [N, 3, H, W] uint8 Spectral."""
    if min_depth >= max_depth:
        raise ValueError(f"Invalid values range: [{min_depth}, {max_depth}].")
    if depth_maps.ndim != 4 or depth_maps.shape[1] != 1:
        raise ValueError(f"Input depth maps must have shape [N,1,H,W], got {depth_maps.shape}")
    d = depth_maps.clamp(min=min_depth, max=max_depth)
    d = ((d - min_depth) / (max_depth - min_depth)).clamp(0.0, 1.0)
    return torch.stack([colormap_spectral(m[0]) for m in d]).permute(0, 3, 1, 2).contiguous()


def make_grid(imgs, nrow: int | None = None, resize: tuple[int, int] | None = None, padding: int = 2) -> torch.Tensor:
    """torchvision.utils.make_grid (padding 2, pad value 0) + optional bilinear resize (utils.py:973-1066)."""
    if isinstance(imgs, list):
        if not imgs:
            raise ValueError("Empty list of images provided")
        imgs = torch.stack([i.cpu() for i in imgs])
    if imgs.dim() != 4:
        raise ValueError("Images must be 4D tensor (N,C,H,W)")
    n, c, h, w = imgs.shape
    nrow = n if nrow is None else nrow
    rows = -(-n // nrow)
    grid = torch.zeros(c, rows * (h + padding) + padding, nrow * (w + padding) + padding, dtype=imgs.dtype)
    for k in range(n):
        y, x = divmod(k, nrow)
        grid[:, y * (h + padding) + padding:y * (h + padding) + padding + h,
             x * (w + padding) + padding:x * (w + padding) + padding + w] = imgs[k]
    if resize is not None:
        th, tw = resize
        if th != -1 or tw != -1:
            _, gh, gw = grid.shape
            th = th if th != -1 else int(tw * gh / gw)
            tw = tw if tw != -1 else int(th * gw / gh)
            g = F.interpolate(grid.unsqueeze(0).float(), size=(th, tw), mode="bilinear", align_corners=False)[0]
            grid = g.round().clamp(0, 255).to(grid.dtype) if grid.dtype == torch.uint8 else g
    return grid


def save_img_tensor(img: torch.Tensor, path: Path) -> None:
    """utils.py:533-589 via torchvision.save_image's rounding: uint8 in, mul(255)+0.5 clamp out."""
    from PIL import Image
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    img = img.detach().cpu()
    if img.dtype == torch.uint8:
        img = img.float() / 255.0
    elif img.dtype == torch.float32:
        if img.max() > 1.0 or img.min() < 0.0:
            raise ValueError("Image tensor must be in the range [0, 1] if dtype is float32")
    else:
        raise ValueError(f"Unsupported image type: {img.dtype}")
    arr = img.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    tmp = _atomic_path(path)
    try:
        Image.fromarray(arr.squeeze(-1) if arr.shape[-1] == 1 else arr).save(tmp)
        os.replace(tmp, path)
    finally:
        if tmp.exists():
            tmp.unlink()

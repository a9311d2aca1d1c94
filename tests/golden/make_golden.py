"""Generate golden vectors by running the REFERENCE's own code (this container only).

``/root/reference`` cannot be imported as a module (``import marigold_dc`` needs
diffusers, ``import utils`` needs blosc2/cv2/torchvision -- ordinary import
errors).  Its pure-torch functions are therefore taken from the
source text with ``ast`` and executed as-is:

* marigold_dc.py: ``get_projection_fn`` (:23), ``compute_affine_params`` (:53),
  ``compute_loss`` (:131) and the methods of ``MarigoldDepthCompletionPipeline``
  (``_affine_to_metric`` :284, ``_latent_to_affine`` :338, ``_latent_to_metric``
  :373, ``_predict_noise`` :432, ``__call__`` :467);
* utils.py: ``kld_stdnorm`` (:28), ``masked_minmax`` (:89).

The reference ``__call__`` runs on top of ``oracle.pipeline_ref.MarigoldBase``,
which supplies the diffusers pieces it inherits (UNet, TAESD, DDIM, image
processor; restated in ``oracle/diffusers_ref.py``).  So these vectors pin the
reference's guidance loop (validation, normalisation, Tweedie preview, affine
fit, loss, backward, grad rescale, Adam, DDIM update, final decode) and its
helper functions; the diffusers modules themselves stay "parity unpinned".

Nothing of the reference is written out -- only input/output tensors.
Run:  python tests/golden/make_golden.py   (writes tests/golden/*.safetensors + meta.json)
"""
from __future__ import annotations

import ast
import json
import sys
from contextlib import nullcontext
from pathlib import Path
from typing import Callable, cast

import torch
from safetensors.torch import save_file
from torch.optim import SGD, Adagrad, Adam, Optimizer

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))

from oracle.diffusers_ref import (AutoencoderTiny, DDIMScheduler, UNet2DConditionModel,  # noqa: E402
                                  synthetic_state_dict, synthetic_taesd_state_dict,
                                  synthetic_text_embedding, tiny_unet_config)
from oracle.pipeline_ref import MarigoldBase  # noqa: E402


def host_fingerprint() -> str:
    """CPU kernels (oneDNN bf16 conv, vectorised libm) differ between host ISAs, so the vectors
    are bit-exact only on a host with the same fingerprint (tests/test_oracle_golden.py)."""
    flags = set()
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("flags"):
                flags = set(line.split(":", 1)[1].split())
                break
    except OSError:
        pass
    isa = [f for f in ("amx_bf16", "avx512_bf16", "avx512f", "avx2") if f in flags]
    return f"torch {torch.__version__} / {torch.backends.cpu.get_cpu_capability()} / {'+'.join(isa)}"


def _extract(path: Path, names: set[str], cls: str | None = None, methods: set[str] | None = None):
    tree = ast.parse(path.read_text())
    funcs, meths = [], []
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in names:
            funcs.append(node)
        if cls and isinstance(node, ast.ClassDef) and node.name == cls:
            for sub in node.body:
                if isinstance(sub, ast.FunctionDef) and sub.name in methods:
                    meths.append(sub)
    return funcs, meths


def load_reference():
    """Return (namespace with the reference's functions, RefPipeline class)."""
    ns: dict = {"torch": torch, "Callable": Callable, "cast": cast, "nullcontext": nullcontext,
                "SGD": SGD, "Adagrad": Adagrad, "Adam": Adam, "Optimizer": Optimizer}
    ufuncs, _ = _extract(REF / "utils.py", {"kld_stdnorm", "masked_minmax", "calc_bins", "mae", "rmse"})
    umod = ast.Module(body=ufuncs, type_ignores=[])
    uns: dict = {"torch": torch}
    exec(compile(umod, str(REF / "utils.py"), "exec"), uns)

    class _Utils:  # stands in for ``import utils`` inside marigold_dc.py
        kld_stdnorm = staticmethod(uns["kld_stdnorm"])
        masked_minmax = staticmethod(uns["masked_minmax"])

    ns["utils"] = _Utils
    src = (REF / "marigold_dc.py").read_text()
    tree = ast.parse(src)
    consts = [n for n in tree.body if isinstance(n, ast.Assign)
              and any(isinstance(t, ast.Name) and t.id in ("SUPPORTED_LOSS_FUNCS", "EPSILON") for t in n.targets)]
    funcs, meths = _extract(REF / "marigold_dc.py", {"get_projection_fn", "compute_affine_params", "compute_loss"},
                            "MarigoldDepthCompletionPipeline",
                            {"_affine_to_metric", "_latent_to_affine", "_latent_to_metric",
                             "_predict_noise", "__call__"})
    mod = ast.Module(body=consts + funcs, type_ignores=[])
    exec(compile(mod, str(REF / "marigold_dc.py"), "exec"), ns)
    cls_body = ast.Module(body=meths, type_ignores=[])
    mns: dict = dict(ns)
    exec(compile(cls_body, str(REF / "marigold_dc.py"), "exec"), mns)
    RefPipeline = type("RefPipeline", (MarigoldBase,), {m.name: mns[m.name] for m in meths})
    return ns, uns, RefPipeline


# ------------------------------------------------------------------ inputs
def synth_inputs(n, h, w, n_points, seed):
    """Seeded synthetic RGB (smooth gradient + noise) and 8-bit-quantised sparse depth."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, h), torch.linspace(0, 1, w), indexing="ij")
    imgs, sparses = [], []
    for i in range(n):
        base = torch.stack([xx, yy, 0.5 * (xx + yy)]) * 200 + 20 * i
        noise = torch.randn((3, h, w), generator=g) * 12
        imgs.append((base + noise).clamp(0, 255).round().to(torch.uint8))
        field = 10 + 80 * yy + 20 * torch.sin(6.28 * xx + i)  # metres
        k = (field * 255 / 120).round().clamp(1, 255)
        sp = torch.zeros(h * w)
        idx = torch.randperm(h * w, generator=g)[:n_points]
        sp[idx] = (120 * k.view(-1)[idx] / 255)
        sparses.append(sp.view(1, h, w))
    return torch.stack(imgs), torch.stack(sparses)


def build_models(dtype, unet_seed=11, vae_seed=12, text_seed=13):
    cfg = tiny_unet_config()
    unet = UNet2DConditionModel(cfg)
    unet.load_state_dict(synthetic_state_dict(unet, unet_seed))
    vae = AutoencoderTiny()
    vae.load_state_dict(synthetic_taesd_state_dict(vae, vae_seed))
    unet.to(dtype)
    vae.to(dtype)
    emb = synthetic_text_embedding(text_seed, cfg.cross_attention_dim)
    return unet, vae, emb


PIPE_CASES = {
    # name: (dtype, n, h, w, res, npts, kwargs)
    "cli_default_bf16": ("bf16", 2, 48, 64, 64, 40, dict(norm="const", steps=3)),
    "cli_default_fp32": ("fp32", 2, 48, 64, 64, 40, dict(norm="const", steps=3)),
    "square_bf16": ("bf16", 1, 64, 64, 64, 30, dict(norm="const", steps=2)),
    "minmax_prev_bf16": ("bf16", 2, 48, 64, 64, 40, dict(norm="minmax", steps=2, beta=0.7, use_prev=True)),
    "closed_form_fp32": ("fp32", 2, 48, 64, 64, 40, dict(norm="const", steps=3, train_latents=False)),
    "per_input_fp32": ("fp32", 1, 48, 64, 64, 40, dict(norm="minmax", steps=2, train_method="per-input",
                                                        train_steps=2)),
    "log_pct_fp32": ("fp32", 1, 48, 64, 64, 40, dict(norm="percentile", steps=2, projection="log10",
                                                      min_depth=1.0)),
    "inv_minmax_fp32": ("fp32", 1, 48, 64, 64, 40, dict(norm="minmax", steps=2, inv=True, min_depth=1.0)),
    "kld_sgd_fp32": ("fp32", 1, 48, 64, 64, 40, dict(norm="const", steps=2, kld=True, opt="sgd",
                                                      loss_funcs=["l1", "l2", "smooth"])),
}


def run_pipe_case(RefPipeline, name, spec):
    dt_name, n, h, w, res, npts, kw = spec
    dtype = torch.bfloat16 if dt_name == "bf16" else torch.float32
    kw = dict(kw)
    use_prev = kw.pop("use_prev", False)
    unet, vae, emb = build_models(dtype)
    pipe = RefPipeline(unet, vae, DDIMScheduler(), emb, dtype=dtype)
    imgs, sparses = synth_inputs(n, h, w, npts, seed=7)
    prev = None
    if use_prev:
        eh, ew = res * h // (8 * max(h, w)), res * w // (8 * max(h, w))
        prev = torch.randn((n, 4, eh, ew), generator=torch.Generator().manual_seed(5)).to(dtype)
    dense, lat = pipe(imgs, sparses, 120.0, resolution=res, pred_latents_prev=prev, **kw)
    out = {"imgs": imgs, "sparses": sparses, "dense": dense.float().contiguous(), "latents": lat.contiguous()}
    if prev is not None:
        out["prev"] = prev.contiguous()
    return out


def make_unit_vectors(ns, uns):
    g = torch.Generator().manual_seed(3)
    n, h, w = 3, 9, 11
    aff = torch.rand((n, 1, h, w), generator=g)
    guide = torch.rand((n, 1, h, w), generator=g) * 2 + 0.5
    mask = torch.rand((n, 1, h, w), generator=g) > 0.6
    img = torch.rand((n, 3, h, w), generator=g)
    lat = torch.randn((n, 4, 5, 6), generator=g)
    out = {"aff": aff, "guide": guide, "mask": mask.to(torch.uint8), "img": img, "lat": lat}
    s, sh = ns["compute_affine_params"](aff, guide, mask)
    out["affine_scale"], out["affine_shift"] = s, sh
    for combo in (["l1"], ["l2"], ["l1", "l2"], ["edge"], ["smooth"]):
        out["loss_" + "_".join(combo)] = ns["compute_loss"](aff, guide, mask, combo, images=img)
    out["loss_kld_simple"] = ns["compute_loss"](aff, guide, mask, ["l1"], images=img, kld=True,
                                                 kld_weight=0.3, kld_mode="simple", pred_latents=lat)
    out["loss_kld_strict"] = ns["compute_loss"](aff, guide, mask, ["l2"], images=img, kld=True,
                                                 kld_weight=0.3, kld_mode="strict", pred_latents=lat)
    mn, mx = uns["masked_minmax"](guide.view(n, -1), mask.view(n, -1), dim=-1)
    out["minmax_min"], out["minmax_max"] = mn, mx
    for p in ("log", "log10", "linear"):
        out["proj_" + p] = ns["get_projection_fn"](p)(guide)
    for red in ("mean", "sum", "none"):
        for mode in ("simple", "strict"):
            out[f"kld_{mode}_{red}"] = uns["kld_stdnorm"](lat, reduction=red, mode=mode).reshape(-1)
    # evaluation helpers of analyze.py (utils.py:162-192, 692-740)
    for name, (lo, hi, size) in {"bins_default": (0.0, 120.0, 10.0), "bins_ragged": (2.5, 100.0, 7.5)}.items():
        out[name] = torch.tensor(uns["calc_bins"](lo, hi, size), dtype=torch.float64)
    dense = torch.rand((n, 1, h, w), generator=g) * 130.0
    sparse = torch.where(mask, (guide * 40).round() * (120.0 / 255.0) * 5, torch.zeros(()))
    out["eval_dense"], out["eval_sparse"] = dense, sparse
    out["eval_mae"] = uns["mae"](dense, sparse, masks=mask).reshape(1)
    out["eval_rmse"] = uns["rmse"](dense, sparse, masks=mask).reshape(1)
    out["eval_mae_nomask"] = uns["mae"](dense, sparse).reshape(1)
    return {k: v.clone().contiguous() for k, v in out.items()}


def main():
    torch.set_num_threads(8)
    ns, uns, RefPipeline = load_reference()
    unit = make_unit_vectors(ns, uns)
    save_file(unit, str(HERE / "unit_functions.safetensors"))
    meta = {"unit_functions": sorted(unit), "host": host_fingerprint()}
    for name, spec in PIPE_CASES.items():
        out = run_pipe_case(RefPipeline, name, spec)
        save_file(out, str(HERE / f"pipe_{name}.safetensors"))
        meta[name] = {"spec": [spec[0], *spec[1:6], {k: v for k, v in spec[6].items()}]}
        print(name, "dense mean", float(out["dense"].mean()))
    (HERE / "meta.json").write_text(json.dumps(meta, indent=1, default=str))


if __name__ == "__main__":
    main()

"""End-to-end parity of the HIP guided sampler against the oracle pipeline (GPU).

The oracle (oracle/pipeline_ref.py, pinned bit-exactly to the reference's own loop code by
tests/test_oracle_golden.py) runs the same synthetic weights, inputs and initial noise.  Parity
statement (tolerances set from measurement): after fitting each dense output to the
sparse points with the reference's closed-form affine (compute_affine_params, marigold_dc.py:53-128),
the per-pixel |depth difference| to the fp32 oracle, relative to the frame's depth range, is at most
2x the oracle's own bf16 execution's (+1e-3), and below mean 2 % / p99 8 % absolute.  With synthetic
weights the bf16 oracle itself sits at ~1.1 % mean / 4.5 % p99 after 10 guided steps, so the survey's
proposed 0.5 % / 2 % is below the bf16 noise floor of the reference path itself.
"""
import pytest
import torch

from oracle import pipeline_ref as P
from oracle.diffusers_ref import (AutoencoderTiny, DDIMScheduler, UNet2DConditionModel, UNetConfig,
                                  synthetic_state_dict, synthetic_taesd_state_dict, synthetic_text_embedding,
                                  tiny_unet_config)

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")
# The oracle legs of the tiny-UNet cases run on the host CPU: deterministic from run to run, so the bf16 leg's error
# (the anchor of every relative bound below) is one fixed number per host, not a sample of PyTorch-ROCm's
# run-to-run spread (its GPU conv backward and SDPA are not deterministic)
ORACLE = torch.device("cpu")


def synth_inputs(n, h, w, n_points, seed):
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, h), torch.linspace(0, 1, w), indexing="ij")
    imgs, sparses = [], []
    for i in range(n):
        base = torch.stack([xx, yy, 0.5 * (xx + yy)]) * 200 + 20 * i
        imgs.append((base + torch.randn((3, h, w), generator=g) * 12).clamp(0, 255).round().to(torch.uint8))
        field = 10 + 80 * yy + 20 * torch.sin(6.28 * xx + i)
        k = (field * 255 / 120).round().clamp(1, 255)
        sp = torch.zeros(h * w)
        idx = torch.randperm(h * w, generator=g)[:n_points]
        sp[idx] = 120 * k.view(-1)[idx] / 255
        sparses.append(sp.view(1, h, w))
    return torch.stack(imgs), torch.stack(sparses)


def fitted_error(dense, ref, sparses):
    """|fit(dense) - fit(ref)| relative to the frame depth range, both fitted to the sparse points."""
    m = sparses > 0
    out = []
    for d in (dense, ref):
        s, sh = P.compute_affine_params(d.float().cpu(), sparses.cpu(), m.cpu())
        out.append(d.float().cpu() * s.view(-1, 1, 1, 1) + sh.view(-1, 1, 1, 1))
    diff = (out[0] - out[1]).abs()
    rng = (out[1].amax(dim=(1, 2, 3)) - out[1].amin(dim=(1, 2, 3))).view(-1, 1, 1, 1)
    r = (diff / rng).flatten(1)
    return float(r.mean()), float(torch.quantile(r.float(), 0.99, dim=1).max())


def build(cfg_o, hcfg, dtype_oracle, dev_o):
    unet = UNet2DConditionModel(cfg_o)
    usd = synthetic_state_dict(unet, 11)
    unet.load_state_dict(usd)
    vae = AutoencoderTiny()
    vsd = synthetic_taesd_state_dict(vae, 12)
    vae.load_state_dict(vsd)
    emb = synthetic_text_embedding(13, cfg_o.cross_attention_dim)
    oracle = P.OracleMarigoldDC(unet.to(dtype_oracle).to(dev_o), vae.to(dtype_oracle).to(dev_o), DDIMScheduler(),
                                emb, dtype=dtype_oracle, device=dev_o)
    return oracle, usd, vsd, emb


@pytest.mark.parametrize("which,n,h,w,res,steps", [("tiny", 2, 48, 64, 64, 10), ("full", 1, 64, 96, 96, 3)])
def test_pipeline_parity(which, n, h, w, res, steps):
    from depth_completion_amd.config import MARIGOLD_V1, TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    cfg_o = tiny_unet_config() if which == "tiny" else UNetConfig()
    hcfg = TINY if which == "tiny" else MARIGOLD_V1
    imgs, sparses = synth_inputs(n, h, w, 60, seed=7)
    eh, ew = -(-(res * h // max(h, w)) // 8), -(-(res * w // max(h, w)) // 8)
    noise = torch.randn((1, 4, eh, ew), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
    kw = dict(norm="const", steps=steps, resolution=res, init_noise=noise)
    od = ORACLE if which == "tiny" else dev
    o32, usd, vsd, emb = build(cfg_o, hcfg, torch.float32, od)
    d32, l32 = o32(imgs.to(od), sparses.to(od), 120.0, **kw)
    o16, *_ = build(cfg_o, hcfg, torch.bfloat16, od)
    d16, l16 = o16(imgs.to(od), sparses.to(od), 120.0, **kw)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=hcfg, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    torch.cuda.synchronize()
    dh, lh, d32, l32, d16, l16 = (t.cpu() for t in (dh, lh, d32, l32, d16, l16))
    assert dh.shape == (n, 1, h, w) and lh.shape == (n, 4, eh, ew) and lh.dtype == torch.bfloat16
    assert torch.isfinite(dh).all()
    mean_h, p99_h = fitted_error(dh, d32, sparses)
    mean_b, p99_b = fitted_error(d16, d32, sparses)
    lat_h = float((lh.float() - l32.float()).norm() / l32.float().norm())
    lat_b = float((l16.float() - l32.float()).norm() / l32.float().norm())
    print(f"\n{which}: HIP fitted |d| mean {mean_h:.5f} p99 {p99_h:.5f} latent {lat_h:.4f} | "
          f"oracle-bf16 mean {mean_b:.5f} p99 {p99_b:.5f} latent {lat_b:.4f}")
    assert mean_h <= 2 * mean_b + 1e-3 and p99_h <= 2 * p99_b + 1e-3
    assert mean_h <= 0.02 and p99_h <= 0.08


def test_graph_replay_matches_eager():
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    cfg_o = tiny_unet_config()
    unet = UNet2DConditionModel(cfg_o)
    usd = synthetic_state_dict(unet, 11)
    vae = AutoencoderTiny()
    vsd = synthetic_taesd_state_dict(vae, 12)
    emb = synthetic_text_embedding(13, cfg_o.cross_attention_dim)
    imgs, sparses = synth_inputs(2, 48, 64, 60, seed=8)
    outs = []
    for use_graph in (False, True, True):  # second graph call re-uses the captured graph
        pipe = outs and use_graph and outs[-1][2] or MarigoldDepthCompletionPipeline(
            usd, vsd, emb, unet_config=TINY, device=dev, use_graph=use_graph)
        d, l = pipe(imgs.to(dev), sparses.to(dev), 120.0, norm="const", steps=6, resolution=64)
        outs.append((d.clone(), l.clone(), pipe))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[1][0], outs[2][0]) and torch.equal(outs[1][1], outs[2][1])


def test_errors_match_reference():
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    cfg_o = tiny_unet_config()
    unet = UNet2DConditionModel(cfg_o)
    vae = AutoencoderTiny()
    pipe = MarigoldDepthCompletionPipeline(synthetic_state_dict(unet, 1), synthetic_taesd_state_dict(vae, 2),
                                           synthetic_text_embedding(3, 64), unet_config=TINY, device=dev)
    imgs, sparses = synth_inputs(1, 48, 64, 60, seed=9)
    with pytest.raises(ValueError):
        pipe(imgs, sparses[:, :, :10], 120.0)
    with pytest.raises(ValueError):
        pipe(imgs, sparses, 120.0, beta=1.5)
    with pytest.raises(ValueError):
        pipe(imgs, sparses, 120.0, projection="sqrt")
    with pytest.raises(ValueError):
        pipe(imgs, sparses, 120.0, closed_form=False, train_latents=False)
    with pytest.raises(ValueError):  # empty mask (utils.py:132-136)
        pipe(imgs, torch.zeros_like(sparses), 120.0, resolution=64, steps=1)


@pytest.mark.parametrize("kw", [dict(norm="const"), dict(norm="minmax", projection="log10", min_depth=1.0),
                                dict(norm="minmax", inv=True, min_depth=1.0)])
def test_plain_ddim_closed_form(kw):
    """train_latents=False: plain DDIM + closed-form affine on the final decode (marigold_dc.py:905-909,
    332-336, 969-985), the mode of the golden case closed_form_fp32 that pins the oracle."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    n, h, w, res, steps = 2, 48, 64, 64, 8
    cfg_o = tiny_unet_config()
    imgs, sparses = synth_inputs(n, h, w, 60, seed=17)
    noise = torch.randn((1, 4, 6, 8), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
    args = dict(kw, steps=steps, resolution=res, init_noise=noise, train_latents=False)
    o32, usd, vsd, emb = build(cfg_o, TINY, torch.float32, ORACLE)
    d32, l32 = o32(imgs, sparses, 120.0, **args)
    o16, *_ = build(cfg_o, TINY, torch.bfloat16, ORACLE)
    d16, l16 = o16(imgs, sparses, 120.0, **args)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **args)
    torch.cuda.synchronize()
    dh, lh = dh.cpu(), lh.cpu()
    assert torch.isfinite(dh).all()
    rng = (d32.amax(dim=(1, 2, 3)) - d32.amin(dim=(1, 2, 3))).view(-1, 1, 1, 1)
    err_h = float(((dh - d32).abs() / rng).mean())
    err_b = float(((d16 - d32).abs() / rng).mean())
    lat_h = float((lh.float() - l32.float()).norm() / l32.float().norm())
    lat_b = float((l16.float() - l32.float()).norm() / l32.float().norm())
    print(f"\nplain DDIM {kw}: HIP |d| {err_h:.5f} latent {lat_h:.4f} | oracle-bf16 |d| {err_b:.5f} latent {lat_b:.4f}")
    assert err_h <= 2 * err_b + 2e-3 and lat_h <= 2 * lat_b + 2e-3


def _mode_parity(args, seed, label, fitted=False, d_factor=2.0, d_abs=0.0):
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    n, h, w, res = 2, 48, 64, 64
    cfg_o = tiny_unet_config()
    imgs, sparses = synth_inputs(n, h, w, 60, seed=seed)
    noise = torch.randn((1, 4, 6, 8), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
    args = dict(args, resolution=res, init_noise=noise)
    o32, usd, vsd, emb = build(cfg_o, TINY, torch.float32, ORACLE)
    d32, l32 = o32(imgs, sparses, 120.0, **args)
    o16, *_ = build(cfg_o, TINY, torch.bfloat16, ORACLE)
    d16, l16 = o16(imgs, sparses, 120.0, **args)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **args)
    torch.cuda.synchronize()
    dh, lh = dh.cpu(), lh.cpu()
    assert torch.isfinite(dh).all() and dh.shape == d32.shape and lh.shape == l32.shape
    lat_h = float((lh.float() - l32.float()).norm() / l32.float().norm())
    lat_b = float((l16.float() - l32.float()).norm() / l32.float().norm())
    if fitted:
        err_h, p99_h = fitted_error(dh, d32, sparses)
        err_b, p99_b = fitted_error(d16, d32, sparses)
    else:
        rng = (d32.amax(dim=(1, 2, 3)) - d32.amin(dim=(1, 2, 3))).view(-1, 1, 1, 1)
        err_h = float(((dh - d32).abs() / rng).mean())
        err_b = float(((d16 - d32).abs() / rng).mean())
    print(f"\n{label}: HIP |d| {err_h:.5f} latent {lat_h:.4f} | oracle-bf16 |d| {err_b:.5f} latent {lat_b:.4f}")
    assert err_h <= max(d_factor * err_b + 2e-3, d_abs) and lat_h <= 2 * lat_b + 2e-3
    return pipe


def test_guided_closed_form():
    """closed_form=True with trainable latents (per-step): the closed-form fit of every preview is part of
    the differentiated loss (marigold_dc.py:332-336 inside :828-877)."""
    _mode_parity(dict(norm="const", steps=8, closed_form=True), 21, "guided closed-form", fitted=True)


@pytest.mark.parametrize("closed_form", [None, True])
def test_per_input(closed_form):
    """train_method="per-input" (marigold_dc.py:911-967): plain DDIM loop, then train_steps optimiser steps
    that move only the learned scale / shift (the optimiser holds the pre-loop latent tensor)."""
    pipe = _mode_parity(dict(norm="minmax", steps=6, train_method="per-input", train_steps=12,
                             closed_form=closed_form), 22, f"per-input closed_form={closed_form}")
    if closed_form is None:
        assert torch.isfinite(pipe.last_loss).all()


@pytest.mark.parametrize("kw", [dict(norm="minmax", projection="log10", min_depth=1.0),
                                dict(norm="const", projection="log", min_depth=2.0),
                                dict(norm="minmax", inv=True, min_depth=1.0),
                                dict(norm="minmax", inv=True, min_depth=1.0, closed_form=True)])
def test_guided_depth_space(kw):
    """Guided steps with the loss in a projected / inverted depth space (marigold_dc.py:843-860)."""
    _mode_parity(dict(kw, steps=6), 23, f"guided {kw}", fitted=True)


def test_per_input_projected():
    _mode_parity(dict(norm="minmax", projection="log", min_depth=1.0, steps=5, train_method="per-input",
                      train_steps=8), 24, "per-input log")


@pytest.mark.parametrize("kw", [dict(opt="sgd", kld=True), dict(opt="adagrad"),
                                dict(kld=True, kld_mode="strict", kld_weight=0.5),
                                dict(opt="sgd", lr=(0.5, 0.05))])
def test_guided_optimisers_kld(kw):
    """Guided steps with SGD / Adagrad (marigold_dc.py:783-789) and the KL term (utils.py:28-86)."""
    _mode_parity(dict(kw, norm="const", steps=6), 25, f"guided {kw}", fitted=True)


@pytest.mark.parametrize("opt", ["sgd", "adagrad"])
def test_per_input_optimisers(opt):
    _mode_parity(dict(norm="minmax", steps=5, train_method="per-input", train_steps=10, opt=opt, lr=(0.05, 0.05)),
                 26, f"per-input {opt}")


@pytest.mark.parametrize("kw", [dict(loss_funcs=["l1", "l2", "edge", "smooth"]),
                                dict(loss_funcs=["l1", "smooth"], norm="minmax"),
                                dict(loss_funcs=["l2", "edge"], projection="log", min_depth=1.0),
                                dict(loss_funcs=["l1"])])
def test_guided_full_image_losses(kw):
    """Guided steps with the edge / smooth terms of compute_loss (marigold_dc.py:195-235) or a single point
    term: the loss runs on the whole dense map (dc_dense_loss)."""
    _mode_parity(dict({"norm": "const"}, **kw, steps=6), 27, f"guided {kw}", fitted=True)


@pytest.mark.parametrize("kw", [dict(), dict(train_latents=False), dict(loss_funcs=["l1", "l2", "smooth"])])
def test_nearest_interp(kw):
    """interp_mode="nearest" for the resize of _latent_to_affine (marigold_dc.py:366-370): the decoded map is
    upsampled 48x64 -> 50x70 here, so the nearest source index differs from bilinear's taps."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    n, h, w, res = 1, 50, 70, 64
    cfg_o = tiny_unet_config()
    imgs, sparses = synth_inputs(n, h, w, 60, seed=28)
    eh, ew = -(-(res * h // max(h, w)) // 8), -(-(res * w // max(h, w)) // 8)
    noise = torch.randn((1, 4, eh, ew), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
    args = dict(kw, norm="const", steps=5, resolution=res, init_noise=noise, interp_mode="nearest")
    o32, usd, vsd, emb = build(cfg_o, TINY, torch.float32, ORACLE)
    d32, l32 = o32(imgs, sparses, 120.0, **args)
    o16, *_ = build(cfg_o, TINY, torch.bfloat16, ORACLE)
    d16, l16 = o16(imgs, sparses, 120.0, **args)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **args)
    torch.cuda.synchronize()
    dh, lh = dh.cpu(), lh.cpu()
    assert dh.shape == d32.shape and torch.isfinite(dh).all()
    err_h, _ = fitted_error(dh, d32, sparses)
    err_b, _ = fitted_error(d16, d32, sparses)
    lat_h = float((lh.float() - l32.float()).norm() / l32.float().norm())
    lat_b = float((l16.float() - l32.float()).norm() / l32.float().norm())
    print(f"\nnearest {kw}: HIP |d| {err_h:.5f} latent {lat_h:.4f} | oracle-bf16 |d| {err_b:.5f} latent {lat_b:.4f}")
    # (the bf16 anchor runs on the host CPU: on PyTorch-ROCm's GPU path its error spread 0.006 - 0.027 between runs,
    # profiles/r04za, which a relative bound cannot take)
    assert err_h <= 2 * err_b + 2e-3 and lat_h <= 2 * lat_b + 2e-3
    # blocky: every output pixel equals one decoded pixel, so the dense map has at most PH*PW levels per frame
    assert dh.unique().numel() <= 48 * 64


@pytest.mark.parametrize("kw", [dict(loss_funcs=["l1", "l2", "edge", "smooth"]), dict(loss_funcs=["l2", "smooth"])])
def test_guided_closed_form_full_image_losses(kw):
    """closed_form=True guided steps with whole-map loss terms: the fit of the preview (compute_affine_params,
    marigold_dc.py:332-336) is differentiated through every pixel's loss (dc_closed_form_stats ->
    dc_dense_loss flag 16 -> dc_closed_form_adjoint).  The scale's gradient sums sign-valued edge / smooth
    terms over every pixel, and the final closed-form fit of a flattened map is ill-conditioned: trajectories
    diverge within a few steps (the oracle's own bf16 run reaches |d| 0.06 after 6 steps and 1.4 after 3 on
    some seeds).  One guided step here, the latent at the usual bound and the final fitted map at 3x; the
    gradient itself is pinned against autograd in tests/test_gpu_guidance.py.  The bf16 oracle's own fitted
    error on these same inputs moves between 0.0098 and 0.032 from run to run (PyTorch-ROCm's conv backward is
    not deterministic; the HIP result is bitwise stable, 0.0361 / 0.0314 for the two loss sets across three
    library builds, profiles/r02o), so the fitted map also passes under an absolute 0.05."""
    _mode_parity(dict({"norm": "const", "closed_form": True}, **kw, steps=1), 30, f"guided cf {kw}", fitted=True,
                 d_factor=3.0, d_abs=0.05)


@pytest.mark.parametrize("kw", [dict(loss_funcs=["l1", "l2", "smooth"]), dict(loss_funcs=["l1", "edge"], opt="sgd")])
def test_per_input_full_image_losses(kw):
    """train_method="per-input" with whole-map loss terms: each of the train_steps optimiser steps of the
    learned scale / shift (marigold_dc.py:911-967, unclamped map) runs dc_dense_loss + dc_affine_step."""
    _mode_parity(dict({"norm": "minmax", "train_method": "per-input", "train_steps": 10}, **kw, steps=5), 31,
                 f"per-input {kw}")


@pytest.mark.parametrize("kw,res", [(dict(), 256), (dict(closed_form=True), 256), (dict(), 192),
                                    (dict(interp_mode="nearest"), 192)])
def test_sparse_aware_decode(kw, res, monkeypatch):
    """Guided steps with the point losses run TAESD's full-resolution layers on the receptive fields of the
    resize taps only (dc_tap_mask / dc_dilate_mask / dc_mask_rows + row-list convs): the result matches the
    dense decode path (DC_SPARSE_DECODE=0) and the oracle.  192x256 images, 40 points: at resolution 256
    the taps are the sparse pixels themselves; at 192 the 144x192 decode is resized up to 192x256, so the
    tap sets come from the bilinear (4 taps) or nearest (1 tap) source rule."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    n, h, w = 1, 192, 256
    ph, pw = -(-(res * h // max(h, w)) // 8) * 8, -(-(res * w // max(h, w)) // 8) * 8
    cfg_o = tiny_unet_config()
    imgs, sparses = synth_inputs(n, h, w, 40, seed=34)
    noise = torch.randn((1, 4, ph // 8, pw // 8), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
    args = dict(kw, norm="const", steps=4, resolution=res, init_noise=noise)
    o32, usd, vsd, emb = build(cfg_o, TINY, torch.float32, ORACLE)
    d32, l32 = o32(imgs, sparses, 120.0, **args)
    o16, *_ = build(cfg_o, TINY, torch.bfloat16, ORACLE)
    d16, l16 = o16(imgs, sparses, 120.0, **args)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DC_SPARSE_DECODE", mode)
        pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
        out[mode] = pipe(imgs.to(dev), sparses.to(dev), 120.0, **args)
        st = pipe._plans[(1, ph // 8, pw // 8)]
        assert (st["graph_key"][-1] != ()) == (mode == "1")   # the row sets were used / not used
    torch.cuda.synchronize()
    (dh, lh), (dd, ld_) = [(a.cpu(), b.cpu()) for a, b in (out["1"], out["0"])]
    lat = lambda a: float((a.float() - l32.float()).norm() / l32.float().norm())  # noqa: E731
    err_h, _ = fitted_error(dh, d32, sparses)
    err_b, _ = fitted_error(d16, d32, sparses)
    print(f"\nsparse decode {kw}: HIP |d| {err_h:.5f} latent {lat(lh):.4f} | dense-decode latent {lat(ld_):.4f} | "
          f"oracle-bf16 |d| {err_b:.5f} latent {lat(l16):.4f}")
    # the two decode paths pick different tiles / K splits (fp32 summation order), so they drift apart as
    # far as two bf16 executions do
    assert float((lh.float() - ld_.float()).norm() / ld_.float().norm()) <= 2 * lat(l16) + 2e-3
    assert err_h <= 2 * err_b + 2e-3 and lat(lh) <= 2 * lat(l16) + 2e-3


def test_invalid_interp_mode():
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    cfg_o = tiny_unet_config()
    unet = UNet2DConditionModel(cfg_o)
    vae = AutoencoderTiny()
    pipe = MarigoldDepthCompletionPipeline(synthetic_state_dict(unet, 1), synthetic_taesd_state_dict(vae, 2),
                                           synthetic_text_embedding(3, 64), unet_config=TINY, device=dev)
    imgs, sparses = synth_inputs(1, 48, 64, 60, seed=9)
    with pytest.raises(ValueError):
        pipe(imgs, sparses, 120.0, resolution=64, steps=1, interp_mode="bicubic")


@pytest.mark.parametrize("kw", [dict(), dict(train_latents=False)])
def test_vae_original(kw):
    """--vae original: the AutoencoderKL encoder (prepare_latents: latent_dist.mode() * 0.18215) and decoder
    (decode_prediction: vae.decode(z / 0.18215)) in the guided loop / the plain DDIM mode, tiny configs."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    from depth_completion_amd.vae_kl import TINY_KL
    from oracle.vae_kl_ref import AutoencoderKL, KLConfig, synthetic_kl_state_dict
    n, h, w, res = 1, 48, 64, 64
    cfg_o = tiny_unet_config()
    imgs, sparses = synth_inputs(n, h, w, 60, seed=29)
    noise = torch.randn((1, 4, 6, 8), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
    args = dict(kw, norm="const", steps=5, resolution=res, init_noise=noise)
    ocfg = KLConfig(block_out_channels=TINY_KL.block_out_channels, layers_per_block=TINY_KL.layers_per_block)
    kl = AutoencoderKL(ocfg)
    ksd = synthetic_kl_state_dict(kl, 31)
    outs = {}
    for dt in (torch.float32, torch.bfloat16):
        unet = UNet2DConditionModel(cfg_o)
        usd = synthetic_state_dict(unet, 11)
        unet.load_state_dict(usd)
        vae = AutoencoderKL(ocfg)
        vae.load_state_dict(ksd)
        emb = synthetic_text_embedding(13, cfg_o.cross_attention_dim)
        o = P.OracleMarigoldDC(unet.to(dt), vae.to(dt), DDIMScheduler(), emb, dtype=dt, device=ORACLE)
        outs[dt] = o(imgs, sparses, 120.0, **args)
    pipe = MarigoldDepthCompletionPipeline(usd, ksd, emb, unet_config=TINY, device=dev, vae="original",
                                           vae_config=TINY_KL)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **args)
    torch.cuda.synchronize()
    dh, lh = dh.cpu(), lh.cpu()
    (d32, l32), (d16, l16) = outs[torch.float32], outs[torch.bfloat16]
    assert dh.shape == d32.shape and torch.isfinite(dh).all()
    err_h, _ = fitted_error(dh, d32, sparses)
    err_b, _ = fitted_error(d16, d32, sparses)
    lat_h = float((lh.float() - l32.float()).norm() / l32.float().norm())
    lat_b = float((l16.float() - l32.float()).norm() / l32.float().norm())
    print(f"\nvae original {kw}: HIP |d| {err_h:.5f} latent {lat_h:.4f} | oracle-bf16 |d| {err_b:.5f} latent {lat_b:.4f}")
    # the VAE mid attention runs materialised (S, P, dP, dS stored in bf16; SDPA keeps them in fp32) and the
    # guided loop's Adam steps amplify that extra rounding: 3x the bf16 oracle's own error in the guided mode
    # (measured: HIP 0.0099 dense / 0.048 latent, bitwise stable, against a bf16 oracle that itself moves
    # between 0.0035 and 0.0041 / 0.014 and 0.022 from run to run -- PyTorch-ROCm's conv backward and SDPA are
    # not deterministic), 2x in the plain DDIM mode
    k = 3 if kw.get("train_latents", True) else 2
    assert err_h <= k * err_b + 2e-3 and lat_h <= k * lat_b + 2e-3


@pytest.mark.parametrize("h,w,npts,density", [(352, 1216, 0, 0.05), (900, 1600, 3000, 0.0)])
def test_baseline_config_shapes(h, w, npts, density):
    """BASELINE.json configs C4 (KITTI 1216x352: resized 222x768, padded to 224 -- latent 28x96 -- and
    unpadded / resized back; 64-beam-like LiDAR rows) and C5 (nuScenes 1600x900: latent 54x96, 3000 points)
    at processing resolution 768 through the tiny UNet, against the oracle."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    g = torch.Generator().manual_seed(30)
    imgs, sparses = synth_inputs(1, h, w, npts, seed=30)
    if density:   # 64 scan rows over the lower 60 % of the image, each pixel kept with p = 0.25
        rows = torch.linspace(0.4 * h, h - 1, 64).round().long()
        keep = torch.zeros(h, w, dtype=torch.bool)
        keep[rows] = torch.rand(64, w, generator=g) < 0.25
        yy, xx = torch.meshgrid(torch.linspace(0, 1, h), torch.linspace(0, 1, w), indexing="ij")
        field = ((10 + 80 * yy + 20 * xx) * 255 / 120).round().clamp(1, 255) * 120 / 255
        sparses = torch.where(keep, field, torch.zeros(()))[None, None]
    res = 768
    eh, ew = -(-(res * h // max(h, w)) // 8), -(-(res * w // max(h, w)) // 8)
    noise = torch.randn((1, 4, eh, ew), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
    args = dict(norm="const", steps=3, resolution=res, init_noise=noise)
    cfg_o = tiny_unet_config()
    o32, usd, vsd, emb = build(cfg_o, TINY, torch.float32, ORACLE)
    d32, l32 = o32(imgs, sparses, 120.0, **args)
    o16, *_ = build(cfg_o, TINY, torch.bfloat16, ORACLE)
    d16, l16 = o16(imgs, sparses, 120.0, **args)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **args)
    torch.cuda.synchronize()
    dh, lh, d32, l32, d16, l16 = (t.cpu() for t in (dh, lh, d32, l32, d16, l16))
    assert dh.shape == (1, 1, h, w) and lh.shape == (1, 4, eh, ew) and torch.isfinite(dh).all()
    err_h, p99_h = fitted_error(dh, d32, sparses)
    err_b, p99_b = fitted_error(d16, d32, sparses)
    lat_h = float((lh.float() - l32.float()).norm() / l32.float().norm())
    lat_b = float((l16.float() - l32.float()).norm() / l32.float().norm())
    print(f"\n{w}x{h}: HIP |d| {err_h:.5f} p99 {p99_h:.5f} latent {lat_h:.4f} | oracle-bf16 |d| {err_b:.5f} "
          f"latent {lat_b:.4f}")
    assert err_h <= 2 * err_b + 2e-3 and lat_h <= 2 * lat_b + 2e-3


def test_graph_cache_step_counts_aba():
    """Plan A (2 frames, 6 steps), plan B (1 frame, 3 steps), plan A again: the second plan-A call replays
    the graph captured in the first, against the time-embedding tables of its step count (kept per step
    count, never freed), and equals a fresh pipeline's call bitwise (plan B's call reallocated
    the tables and plan A's graph replayed the freed address)."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    cfg_o = tiny_unet_config()
    unet = UNet2DConditionModel(cfg_o)
    usd = synthetic_state_dict(unet, 11)
    vsd = synthetic_taesd_state_dict(AutoencoderTiny(), 12)
    emb = synthetic_text_embedding(13, cfg_o.cross_attention_dim)
    imgs, sparses = synth_inputs(2, 48, 64, 60, seed=8)
    a = dict(norm="const", steps=6, resolution=64)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    pipe(imgs.to(dev), sparses.to(dev), 120.0, **a)
    g_a = pipe._plans[(2, 6, 8)]["graph"]
    pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **dict(a, steps=3))
    torch.cuda.empty_cache()
    junk = torch.full((1 << 22,), 7.0, device=dev)   # recycle freed blocks with garbage
    d1, l1 = pipe(imgs.to(dev), sparses.to(dev), 120.0, **a)
    assert pipe._plans[(2, 6, 8)]["graph"] is g_a   # replayed, not recaptured
    fresh = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    d2, l2 = fresh(imgs.to(dev), sparses.to(dev), 120.0, **a)
    torch.cuda.synchronize()
    del junk
    assert torch.equal(d1, d2) and torch.equal(l1, l2)


def test_graph_replay_new_frames_same_bucket():
    """Frame set A, then frame set B (other sparse points, same count, same row bucket) on one pipeline at
    resolution 256 with the sparse-aware decode: B's call replays A's captured step graph with the tables and
    decode row lists refreshed in place, and equals a fresh pipeline's run on B bitwise."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    cfg_o = tiny_unet_config()
    usd = synthetic_state_dict(UNet2DConditionModel(cfg_o), 11)
    vsd = synthetic_taesd_state_dict(AutoencoderTiny(), 12)
    emb = synthetic_text_embedding(13, cfg_o.cross_attention_dim)
    ia, sa = synth_inputs(2, 192, 256, 40, seed=60)
    ib, sb = synth_inputs(2, 192, 256, 40, seed=61)
    assert not torch.equal(sa, sb)
    kw = dict(norm="const", steps=4, resolution=256)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    pipe(ia.to(dev), sa.to(dev), 120.0, **kw)
    st = pipe._plans[(2, 24, 32)]
    g_a, key_a = st["graph"], st["graph_key"]
    assert key_a[-1] != ()                       # the sparse-aware decode row lists are in use
    db, lb = pipe(ib.to(dev), sb.to(dev), 120.0, **kw)
    assert st["graph"] is g_a and st["graph_key"] == key_a   # replayed, not recaptured
    fresh = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    df, lf = fresh(ib.to(dev), sb.to(dev), 120.0, **kw)
    torch.cuda.synchronize()
    assert torch.equal(db, df) and torch.equal(lb, lf)


def test_side_stream_shortcuts_bitwise(monkeypatch):
    """DC_SIDE_STREAM=1 (the resnet shortcut convs as a concurrent branch of the captured step graph, their own stream
    and workspace; off by default, measured slower, profiles/r06p) gives the single-stream results bit for bit: the
    same kernels on the same operands, only the launch order differs."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    n, h, w = 1, 192, 256
    cfg_o = tiny_unet_config()
    imgs, sparses = synth_inputs(n, h, w, 40, seed=35)
    _, usd, vsd, emb = build(cfg_o, TINY, torch.float32, ORACLE)
    args = dict(norm="const", steps=4, resolution=256)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DC_SIDE_STREAM", mode)
        pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
        d, lat = pipe(imgs.to(dev), sparses.to(dev), 120.0, **args)
        torch.cuda.synchronize()
        out[mode] = (d.cpu(), lat.cpu())
        assert all((st["unet"].side is not None) == (mode == "1") for st in pipe._plans.values())
    assert torch.equal(out["0"][0], out["1"][0])
    assert torch.equal(out["0"][1].view(torch.int16), out["1"][1].view(torch.int16))

"""The CPU oracle (oracle/) against golden vectors produced by running the reference's own code.

Golden files: tests/golden/*.safetensors, made by tests/golden/make_golden.py, which executes
marigold_dc.py / utils.py functions (AST-extracted) on top of the restated diffusers modules.
A bit-exact match here pins the oracle's restatement of marigold_dc.py:467-985 and utils.py:28-138.
"""
import json
import sys
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

from oracle import pipeline_ref as P
from oracle.diffusers_ref import (AutoencoderTiny, DDIMScheduler, UNet2DConditionModel, synthetic_state_dict,
                                  synthetic_taesd_state_dict, synthetic_text_embedding, tiny_unet_config)

GOLD = Path(__file__).resolve().parent / "golden"


def _same(got, exp):
    """Bit-exact up to a couple of fp32 ulps: torch's vectorised log/exp differ by 1 ulp between
    host ISAs (the goldens were made on an AVX-512 Xeon; the suite also runs on EPYC hosts)."""
    torch.testing.assert_close(got, exp, rtol=3e-7, atol=1e-7)


def test_unit_functions_match_reference():
    u = load_file(str(GOLD / "unit_functions.safetensors"))
    aff, guide, mask, img, lat = u["aff"], u["guide"], u["mask"].bool(), u["img"], u["lat"]
    s, sh = P.compute_affine_params(aff, guide, mask)
    _same(s, u["affine_scale"])
    _same(sh, u["affine_shift"])
    for combo in (["l1"], ["l2"], ["l1", "l2"], ["edge"], ["smooth"]):
        got = P.compute_loss(aff, guide, mask, combo, images=img)
        _same(got, u["loss_" + "_".join(combo)])
    got = P.compute_loss(aff, guide, mask, ["l1"], images=img, kld=True, kld_weight=0.3, kld_mode="simple",
                         pred_latents=lat)
    _same(got, u["loss_kld_simple"])
    got = P.compute_loss(aff, guide, mask, ["l2"], images=img, kld=True, kld_weight=0.3, kld_mode="strict",
                         pred_latents=lat)
    _same(got, u["loss_kld_strict"])
    mn, mx = P.masked_minmax(guide.view(3, -1), mask.view(3, -1), dim=-1)
    _same(mn, u["minmax_min"])
    _same(mx, u["minmax_max"])
    for p in ("log", "log10", "linear"):
        _same(P.get_projection_fn(p)(guide), u["proj_" + p])
    from oracle import analyze_ref as A
    assert torch.equal(torch.tensor(A.calc_bins(0.0, 120.0, 10.0), dtype=torch.float64), u["bins_default"])
    assert torch.equal(torch.tensor(A.calc_bins(2.5, 100.0, 7.5), dtype=torch.float64), u["bins_ragged"])
    d, sp = u["eval_dense"], u["eval_sparse"]
    _same(A.mae(d, sp, masks=mask).reshape(1), u["eval_mae"])
    _same(A.rmse(d, sp, masks=mask).reshape(1), u["eval_rmse"])
    _same(A.mae(d, sp).reshape(1), u["eval_mae_nomask"])
    for red in ("mean", "sum", "none"):
        for mode in ("simple", "strict"):
            _same(P.kld_stdnorm(lat, reduction=red, mode=mode).reshape(-1), u[f"kld_{mode}_{red}"])


def test_error_behaviour():
    with pytest.raises(ValueError):
        P.masked_minmax(torch.ones(2, 3), torch.zeros(2, 3, dtype=torch.bool), dim=-1)
    with pytest.raises(ValueError):
        P.compute_affine_params(torch.ones(1, 1, 2, 2), torch.ones(1, 1, 2, 2), torch.zeros(1, 1, 2, 2))
    with pytest.raises(ValueError):
        P.get_projection_fn("sqrt")
    with pytest.raises(ValueError):
        P.compute_loss(torch.ones(1, 1, 2, 2), torch.ones(1, 1, 2, 2), torch.ones(1, 1, 2, 2), [])


def _build(dtype):
    cfg = tiny_unet_config()
    unet = UNet2DConditionModel(cfg)
    unet.load_state_dict(synthetic_state_dict(unet, 11))
    vae = AutoencoderTiny()
    vae.load_state_dict(synthetic_taesd_state_dict(vae, 12))
    unet.to(dtype)
    vae.to(dtype)
    return P.OracleMarigoldDC(unet, vae, DDIMScheduler(), synthetic_text_embedding(13, cfg.cross_attention_dim),
                              dtype=dtype)


META = json.loads((GOLD / "meta.json").read_text())
CASES = [k for k in META if k not in ("unit_functions", "host")]
sys.path.insert(0, str(GOLD))
from make_golden import host_fingerprint  # noqa: E402

SAME_HOST = META.get("host") == host_fingerprint()


@pytest.mark.parametrize("case", CASES)
def test_pipeline_matches_reference_loop(case):
    torch.set_num_threads(min(8, torch.get_num_threads()))
    g = load_file(str(GOLD / f"pipe_{case}.safetensors"))
    dt, n, h, w, res, npts, kw = META[case]["spec"]
    dtype = torch.bfloat16 if dt == "bf16" else torch.float32
    kw = dict(kw)
    kw.pop("use_prev", None)
    pipe = _build(dtype)
    dense, lat = pipe(g["imgs"], g["sparses"], 120.0, resolution=res, pred_latents_prev=g.get("prev"), **kw)
    if SAME_HOST:
        # Same CPU ops in the same order: bit-exact in practice.  A small tolerance covers the
        # reference's own run-to-run jitter from multithreaded CPU reductions (seen at ~3e-7).
        torch.testing.assert_close(lat.float(), g["latents"].float(), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(dense.float(), g["dense"], rtol=1e-5, atol=1e-4)
        return
    # Vectors made on a host with another CPU ISA: the reference itself moves by this much
    # between an AMX Xeon and an AVX512-bf16 EPYC (bf16: 4.4 % latent / 0.8 % dense relative
    # norm after 3 guided steps; fp32: 1.7e-5 / 1.4e-6), so only a cross-host bound is meaningful.
    tol_lat, tol_dense = (0.1, 0.02) if dtype == torch.bfloat16 else (1e-4, 1e-5)
    for got, exp, tol in ((lat, g["latents"], tol_lat), (dense, g["dense"], tol_dense)):
        got, exp = got.float(), exp.float()
        assert float((got - exp).norm() / exp.norm()) < tol

"""Host-side (CPU) pieces of the library and of the construction surface (no GPU needed).

* dc_schedule_tables / dc_timestep_embedding / dc_fold_cross_attention -- the CPU code both hosts (Python pipeline
  and native session) feed the kernels with -- against the torch formulas of the reference path (DDIMScheduler
  trailing, torch.optim.Adam, diffusers get_timestep_embedding, the attn2 fold of weights.py's docstring);
* the CLIP empty-prompt embedding restatement (pretrained.clip_empty_prompt_embedding) against transformers'
  CLIPTextModel with the same random weights (an independent implementation; marigold_dc.py:663-674);
* the diffusers-layout directory round trip and the scheduler-config check of from_pretrained.
"""
import json
import math

import numpy as np
import pytest
import torch

from depth_completion_amd import pretrained as pt
from depth_completion_amd.config import TINY
from depth_completion_amd.pipeline import DDIM_CONFIG, DDIMTables, adam_table
from depth_completion_amd.unet import timestep_embedding
from depth_completion_amd.weights import fold_cross_attention


def _torch_ddim(steps, T=1000):
    betas = torch.linspace(0.00085 ** 0.5, 0.012 ** 0.5, T, dtype=torch.float32) ** 2
    ac = torch.cumprod(1.0 - betas, dim=0)
    ts = np.round(np.arange(T, 0, -T / steps)).astype(np.int64) - 1
    rows = []
    for t in ts:
        a = ac[t]
        prev = int(t) - T // steps
        ap = ac[prev] if prev >= 0 else ac[0]
        rows.append(torch.stack([a ** 0.5, (1 - a) ** 0.5, ap ** 0.5, (1 - ap) ** 0.5]))
    return torch.from_numpy(ts), torch.stack(rows).float()


@pytest.mark.parametrize("steps", [1, 3, 4, 10, 50])
def test_schedule_tables_match_torch_ddim(steps):
    ts, coef = _torch_ddim(steps)
    d = DDIMTables()
    assert torch.equal(d.timesteps(steps), ts)
    # torch's vectorised linspace rounds some betas one ulp apart from the scalar formula
    torch.testing.assert_close(d.coef(steps), coef, rtol=2e-7, atol=2e-7)
    if steps == 50:
        assert ts[0] == 999 and ts[-1] == 19 and torch.equal(ts[:-1] - ts[1:], torch.full((49,), 20))


def test_adam_table_is_torch_adam_bias_correction():
    tab = adam_table(50, 0.05, 0.005)
    for k in (1, 2, 25, 50):
        bc1, bc2 = 1 - 0.9 ** k, 1 - 0.999 ** k
        assert tab[k - 1].tolist() == torch.tensor([0.05 / bc1, bc2 ** 0.5, 0.005 / bc1, 0.0], dtype=torch.float32).tolist()
    sgd = adam_table(5, 0.05, 0.005, opt=1)
    assert torch.equal(sgd, torch.tensor([[0.05, 0.0, 0.005, 0.0]] * 5, dtype=torch.float32))


def test_timestep_embedding_matches_diffusers_formula():
    ts = DDIMTables().timesteps(50)
    dim = 320
    half = dim // 2
    exponent = -math.log(10000) * torch.arange(0, half, dtype=torch.float32) / half
    emb = ts[:, None].float() * torch.exp(exponent)[None, :]
    ref = torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1)
    # |arg| up to ~1e3 rad: one ulp of exp() moves sin / cos by up to ~1e-4
    torch.testing.assert_close(timestep_embedding(ts, dim), ref, rtol=0, atol=2e-4)


def test_fold_cross_attention_matches_attn2_on_two_tokens():
    """U / D / c0 against an explicit 2-key softmax attention in double (one row of queries)."""
    g = torch.Generator().manual_seed(4)
    C, cross, heads = 64, 32, 2
    hd = C // heads
    sd = {"to_q.weight": torch.randn(C, C, generator=g) * 0.1, "to_k.weight": torch.randn(C, cross, generator=g) * 0.1,
          "to_v.weight": torch.randn(C, cross, generator=g) * 0.1,
          "to_out.0.weight": torch.randn(C, C, generator=g) * 0.1, "to_out.0.bias": torch.randn(C, generator=g) * 0.1}
    ctx = torch.randn(2, cross, generator=g)
    U, D, c0 = fold_cross_attention(sd, "", ctx, heads)
    r = {k: v.bfloat16().double() for k, v in sd.items()}
    c = ctx.bfloat16().double()
    k = (c @ r["to_k.weight"].t()).float().bfloat16().double()
    v = (c @ r["to_v.weight"].t()).float().bfloat16().double()
    x = torch.randn(5, C, generator=g, dtype=torch.float64)
    q = x @ r["to_q.weight"].t()
    out = []
    for h in range(heads):
        sl = slice(h * hd, (h + 1) * hd)
        p = torch.softmax(q[:, sl] @ k[:, sl].t() / math.sqrt(hd), dim=-1)
        out.append(p @ v[:, sl])
    ref = torch.cat(out, -1) @ r["to_out.0.weight"].t() + r["to_out.0.bias"]
    folded = c0.double() + torch.sigmoid(x @ U.double().t()) @ D.double()
    torch.testing.assert_close(folded, ref, rtol=1e-6, atol=1e-6)


def test_fold_layernorm_matches_definition():
    """dc_fold_layernorm (weights.LnLinear, shared with the native session): wf = bf16(W diag(gamma)),
    csum = row sums of wf, cbias = W . beta + bias; LayerNorm(x) @ W^T + bias == rstd (x @ wf^T - mean csum) + cbias
    in exact arithmetic, up to bf16 rounding of the folded weight."""
    from depth_completion_amd.weights import LnLinear, round_bf16
    g = torch.Generator().manual_seed(5)
    n, k = 48, 64
    w = torch.randn(n, k, generator=g)
    b = torch.randn(n, generator=g) * 0.1
    gam = 1 + 0.2 * torch.randn(k, generator=g)
    bet = 0.2 * torch.randn(k, generator=g)
    lin = LnLinear(w, b, gam, bet, 1e-5, "cpu")
    wr, gr, br, bb = round_bf16(w), round_bf16(gam), round_bf16(bet), round_bf16(b)
    assert torch.equal(lin.wf, (wr * gr).to(torch.bfloat16))
    assert torch.equal(lin.wd, lin.wf.t())
    torch.testing.assert_close(lin.csum.double(), lin.wf.double().sum(1), rtol=1e-7, atol=1e-9)
    torch.testing.assert_close(lin.cbias.double(), wr.double() @ br.double() + bb.double(), rtol=1e-7, atol=1e-9)
    x = torch.randn(5, k, generator=g) * 3 + 2
    mu = x.mean(1, keepdim=True)
    rs = torch.rsqrt(x.var(1, unbiased=False, keepdim=True) + 1e-5)
    ref = torch.nn.functional.layer_norm(x, (k,), gr, br, 1e-5) @ wr.t() + bb
    got = rs * (x @ lin.wf.float().t() - mu * lin.csum) + lin.cbias
    assert float((got - ref).norm() / ref.norm()) < 1e-2


def test_clip_empty_prompt_matches_transformers():
    transformers = pytest.importorskip("transformers")
    cfg = transformers.CLIPTextConfig(vocab_size=49408, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                      num_attention_heads=4, max_position_embeddings=77, hidden_act="gelu",
                                      layer_norm_eps=1e-5)
    torch.manual_seed(0)
    model = transformers.CLIPTextModel(cfg).eval()
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    ids = torch.tensor([[pt.BOS, pt.EOS]])
    with torch.no_grad():
        ref = model(ids)[0]
    ours = pt.clip_empty_prompt_embedding(sd, cfg.to_dict())
    torch.testing.assert_close(ours, ref, rtol=1e-5, atol=1e-5)


def test_pretrained_dir_round_trip_and_scheduler_check(tmp_path):
    from depth_completion_amd import synthetic
    usd = synthetic.unet_state_dict(TINY, 11)
    emb = synthetic.text_embedding(13, TINY.cross_attention_dim)
    d = pt.save_pretrained(tmp_path / "ckpt", usd, TINY, taesd_state=synthetic.taesd_state_dict(12),
                           text_embedding=emb)
    u = pt.UNet2DConditionModel.from_pretrained(d)
    assert u.unet_config() == TINY
    assert set(u.state_dict) == set(usd) and torch.equal(u.state_dict["conv_in.weight"], usd["conv_in.weight"])
    assert torch.equal(pt.empty_text_embedding(d), emb.reshape(1, -1, emb.shape[-1]).float())
    shipped = pt.DDIMScheduler.from_pretrained(d)
    assert shipped.config["timestep_spacing"] == "leading"
    with pytest.raises(ValueError, match="timestep_spacing"):
        DDIMTables(shipped.config).coef(10)
    swapped = pt.DDIMScheduler.from_config(shipped.config, timestep_spacing="trailing")
    assert torch.equal(DDIMTables(swapped.config).coef(10), DDIMTables().coef(10))
    assert json.loads((d / "unet" / "config.json").read_text())["attention_head_dim"] == list(TINY.heads)
    with pytest.raises(ValueError):
        pt.AutoencoderTiny.from_pretrained(d / "taesd", torch_dtype=torch.float32)
    assert DDIM_CONFIG["prediction_type"] == "v_prediction"


def test_text_embedding_computed_from_text_encoder(tmp_path):
    from depth_completion_amd import synthetic
    te = pt.synthetic_clip_state(64, 2, 128)
    d = pt.save_pretrained(tmp_path / "ckpt", synthetic.unet_state_dict(TINY, 11), TINY,
                           taesd_state=synthetic.taesd_state_dict(12), text_encoder_state=te,
                           text_encoder_config={"hidden_size": 64, "num_attention_heads": 4, "num_hidden_layers": 2,
                                                "hidden_act": "gelu", "layer_norm_eps": 1e-5})
    emb = pt.empty_text_embedding(d)
    assert emb.shape == (1, 2, 64) and torch.isfinite(emb).all()
    assert (d / "empty_text_embedding.safetensors").exists()   # cached for the native session
    assert torch.equal(pt.empty_text_embedding(d), emb)


def test_conv_pick_exact_nearest_and_filters():
    """dc_conv_pick (both hosts' GEMM variant choice): exact key first; else the nearest tuned shape with the same
    (mode, kh, stride, two_sources) in 4|dlog2 M| + |dlog2 N| + |dlog2 K|, first in table order on ties."""
    from depth_completion_amd.ops import pick_variant
    base = (0, 1, 72, 96, 320, 72, 96, 320, 3, 1, False, 2880)      # M 6912, N 320, K 2880
    table = [(base, (13, -3)),
             ((0, 1, 18, 24, 1280, 18, 24, 1280, 3, 1, False, 11520), (3, 2)),   # M 432
             ((0, 1, 1, 6912, 320, 1, 6912, 320, 1, 1, False, 320), (18, 4)),    # 1x1, other kh
             ((0, 1, 72, 96, 640, 72, 96, 320, 3, 1, True, 5760), (10, 1)),     # two sources
             ((0, 8, 72, 96, 320, 72, 96, 320, 3, 1, False, 2880), (6, 1))]     # M 55296
    assert pick_variant(table, base) == (13, -3)
    assert pick_variant(table, (0, 1, 28, 96, 320, 28, 96, 320, 3, 1, False, 2880)) == (13, -3)   # M 2688
    assert pick_variant(table, (0, 1, 9, 12, 1280, 9, 12, 1280, 3, 1, False, 11520)) == (3, 2)     # M 108
    assert pick_variant(table, (0, 4, 72, 96, 320, 72, 96, 320, 3, 1, False, 2880)) == (6, 1)      # M 27648
    assert pick_variant(table, (0, 1, 1, 2688, 320, 1, 2688, 320, 1, 1, False, 320)) == (18, 4)    # only 1x1 entry
    assert pick_variant(table, (0, 1, 28, 96, 640, 28, 96, 320, 3, 1, True, 5760)) == (10, 1)      # two-source filter
    assert pick_variant(table, (1, 1, 28, 96, 320, 56, 192, 320, 3, 1, False, 2880)) == (0, 0)     # no mode-1 entry
    tie = [((0, 1, 1, 100, 64, 1, 100, 64, 1, 1, False, 64), (1, 1)), ((0, 1, 1, 400, 64, 1, 400, 64, 1, 1, False, 64),
                                                                      (2, 1))]
    assert pick_variant(tie, (0, 1, 1, 200, 64, 1, 200, 64, 1, 1, False, 64)) == (1, 1)            # tie: first
    assert pick_variant([], base) == (0, 0)


@pytest.mark.parametrize("c,k2", [(64, 256), (320, 1280)])
def test_fold_linear_pair_matches_fp64(c, k2):
    """dc_fold_linear_pair (FF2 + proj_out folded into one linear over [gg | r2]) against fp64 torch: wf = [Wp W2 | Wp]
    rounded to bf16, wd = wf^T exactly, bias = Wp b2 + bp; and the folded linear gives the two linears' output."""
    from depth_completion_amd.weights import FoldedPair
    g = torch.Generator().manual_seed(5)
    w2 = (torch.randn(c, k2, generator=g) / k2 ** 0.5).to(torch.bfloat16).float()
    wp = (torch.randn(c, c, generator=g) / c ** 0.5).to(torch.bfloat16).float()
    b2 = (torch.randn(c, generator=g) * 0.1).to(torch.bfloat16).float()
    bp = (torch.randn(c, generator=g) * 0.1).to(torch.bfloat16).float()
    f = FoldedPair(w2, b2, wp, bp, "cpu")
    wref = (wp.double() @ w2.double()).to(torch.bfloat16)
    assert f.wf.shape == (c, k2 + c) and f.wd.shape == (k2 + c, c)
    # (fp64 sums in another order, and the fold's double -> fp32 -> bf16 rounding: a rare tie rounds one ulp apart)
    diff = (f.wf[:, :k2] != wref)
    assert float(diff.float().mean()) < 1e-3
    torch.testing.assert_close(f.wf[:, :k2].float(), wref.float(), rtol=8e-3, atol=1e-7)
    assert torch.equal(f.wf[:, k2:], wp.to(torch.bfloat16))
    assert torch.equal(f.wd, f.wf.t().contiguous())
    torch.testing.assert_close(f.bias.double(), wp.double() @ b2.double() + bp.double(), rtol=1e-6, atol=1e-6)
    gg = torch.randn(7, k2, generator=g).double()
    r2 = torch.randn(7, c, generator=g).double()
    two = ((gg @ w2.double().t() + b2.double() + r2) @ wp.double().t()) + bp.double()
    one = torch.cat([gg, r2], 1) @ f.wf.double().t() + f.bias.double()
    assert float((one - two).norm() / two.norm()) < 1e-2

"""Model-level parity on the GPU: the HIP UNet / TAESD (forward and input-gradient) against the
CPU-restated diffusers modules of ``oracle/`` run with autograd.

Bar: the HIP path (bf16 storage, fp32 accumulation) must be as close to the fp32 oracle as the
oracle's own bf16 execution is: err(HIP, fp32) <= 2 * err(oracle-bf16, fp32) + 2e-3.
"""
import pytest
import torch

from oracle.diffusers_ref import (AutoencoderTiny, UNet2DConditionModel, synthetic_state_dict,
                                  synthetic_taesd_state_dict, synthetic_text_embedding, tiny_unet_config)
from oracle.diffusers_ref import UNetConfig as OracleUNetConfig

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def to_nhwc(x):
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c)


def from_nhwc(t, n, h, w, c):
    return t[:, :c].float().reshape(n, h, w, c).permute(0, 3, 1, 2)


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from depth_completion_amd.ops import Ctx
    return Ctx(dev)


def _oracle_unet_grads(unet, x8, t, emb, dv, dtype):
    m = unet.to(dtype)
    x = x8.to(dtype).clone().requires_grad_(True)
    # _predict_noise repeats the empty-prompt embedding per frame (marigold_dc.py:463)
    v = m(x, torch.tensor(t, device=dev), emb.to(dtype).repeat(x.shape[0], 1, 1))[0]
    v.backward(dv.to(dtype))
    return v.float().detach(), x.grad[:, 4:8].float()


@pytest.mark.parametrize("cfgname,n,h,w,t", [("tiny", 2, 16, 16, 999), ("tiny", 1, 6, 8, 519),
                                              ("full", 1, 8, 12, 19)])
def test_unet_forward_backward(ctx, monkeypatch, cfgname, n, h, w, t):
    from depth_completion_amd.config import MARIGOLD_V1, TINY
    from depth_completion_amd.unet import UNetHIP
    ocfg = tiny_unet_config() if cfgname == "tiny" else OracleUNetConfig()
    hcfg = TINY if cfgname == "tiny" else MARIGOLD_V1
    oracle = UNet2DConditionModel(ocfg)
    sd = synthetic_state_dict(oracle, 11)
    oracle.load_state_dict(sd)
    oracle = oracle.to(torch.bfloat16).float().to(dev)  # bf16-valued weights in fp32
    emb = synthetic_text_embedding(13, ocfg.cross_attention_dim).to(dev)
    g = torch.Generator().manual_seed(1)
    x8 = torch.randn(n, 8, h, w, generator=g).to(torch.bfloat16).float().to(dev)
    dv = torch.randn(n, 4, h, w, generator=g).to(torch.bfloat16).float().to(dev)
    v32, gx32 = _oracle_unet_grads(oracle, x8, t, emb, dv, torch.float32)
    oracle_b = UNet2DConditionModel(ocfg)
    oracle_b.load_state_dict(sd)
    v16, gx16 = _oracle_unet_grads(oracle_b.to(dev), x8, t, emb, dv, torch.bfloat16)

    net = UNetHIP({k: v.float() for k, v in sd.items()}, hcfg, dev, emb.cpu())
    net.build_temb_tables(ctx, torch.tensor([t]))
    ctx.step.zero_()
    plan = net.plan(ctx, n, h, w)
    plan.x8.copy_(to_nhwc(x8).to(torch.bfloat16))
    plan.dv.zero_()
    plan.dv[:, :4].copy_(to_nhwc(dv).to(torch.bfloat16))
    plan.forward()
    plan.backward()
    torch.cuda.synchronize()
    v_h = from_nhwc(plan.v, n, h, w, 4)
    g_h = from_nhwc(plan.gx, n, h, w, 4)
    ev, ev16 = rel(v_h, v32), rel(v16, v32)
    eg, eg16 = rel(g_h, gx32), rel(gx16, gx32)
    print(f"\n{cfgname} {n}x{h}x{w}: v err {ev:.4f} (oracle bf16 {ev16:.4f}); grad err {eg:.4f} (oracle bf16 {eg16:.4f})")
    assert ev <= 2 * ev16 + 2e-3
    assert eg <= 2 * eg16 + 2e-3
    # the separate GroupNorm statistics passes (DC_GN_FUSE=0) against the fused default: the same math up to the
    # statistics' summation (exact sums vs fp32 partials), so bf16 rounding flips only
    monkeypatch.setenv("DC_GN_FUSE", "0")
    plan2 = net.plan(ctx, n, h, w)
    assert not plan2.fuse_gn and plan.fuse_gn
    plan2.x8.copy_(plan.x8)
    plan2.dv.copy_(plan.dv)
    plan2.forward()
    plan2.backward()
    torch.cuda.synchronize()
    v_s, g_s = from_nhwc(plan2.v, n, h, w, 4), from_nhwc(plan2.gx, n, h, w, 4)
    ev2, eg2 = rel(v_s, v_h), rel(g_s, g_h)
    evs, egs = rel(v_s, v32), rel(g_s, gx32)
    print(f"separate statistics: v err {evs:.4f}, grad err {egs:.4f}; fused vs separate: v {ev2:.5f}, grad {eg2:.5f}")
    assert evs <= 2 * ev16 + 2e-3 and egs <= 2 * eg16 + 2e-3
    # both within the bf16 noise floor of each other (the tiny random-weight UNet amplifies one-ulp differences
    # in the statistics of its 2- and 4-channel groups into percent-level output changes, like any bf16 rounding)
    assert ev2 <= max(ev16, 2e-3) and eg2 <= max(eg16, 2e-3)


def test_taesd_decoder_encoder(ctx):
    from depth_completion_amd import ops
    from depth_completion_amd.taesd import TAESDHIP
    vae = AutoencoderTiny()
    sd = synthetic_taesd_state_dict(vae, 12)
    vae.load_state_dict(sd)
    vae32 = vae.to(torch.bfloat16).float().to(dev)
    n, h, w = 2, 6, 8
    g = torch.Generator().manual_seed(2)
    z = torch.randn(n, 4, h, w, generator=g).to(torch.bfloat16).float().to(dev)
    # oracle: out = layers(tanh(z/3)*3), grad w.r.t. the clamp output; fp32 and bf16 executions
    zc = (torch.tanh(z / 3) * 3).to(torch.bfloat16).float().detach().requires_grad_(True)
    out = vae32.decoder.layers(zc)
    gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16).float().to(dev)
    out.backward(gout)
    vae16 = AutoencoderTiny()
    vae16.load_state_dict(sd)
    vae16 = vae16.to(torch.bfloat16).to(dev)
    zc16 = zc.detach().to(torch.bfloat16).requires_grad_(True)
    out16 = vae16.decoder.layers(zc16)
    out16.backward(gout.to(torch.bfloat16))
    e_out16, e_g16 = rel(out16, out), rel(zc16.grad, zc.grad)
    net = TAESDHIP({k: v.float() for k, v in sd.items()}, dev)
    dp = net.decoder_plan(ctx, n, h, w)
    zc_b = to_nhwc(zc.detach()).to(torch.bfloat16)
    dp.tin.zero_()
    dp.tin[:, :4].copy_(zc_b)
    dp.forward()
    dp.dout.zero_()
    dp.dout[:, :3].copy_(to_nhwc(gout).to(torch.bfloat16))
    dp.backward()
    torch.cuda.synchronize()
    H, W = 8 * h, 8 * w
    e_out = rel(from_nhwc(dp.out, n, H, W, 3), out)
    e_g = rel(from_nhwc(dp.dtin, n, h, w, 4), zc.grad)
    print(f"\ntaesd dec out err {e_out:.4f} (oracle bf16 {e_out16:.4f}) grad err {e_g:.4f} (oracle bf16 {e_g16:.4f})")
    assert e_out <= 2 * e_out16 + 2e-3 and e_g <= 2 * e_g16 + 2e-3
    # encoder on a [0,1] image
    img = torch.rand(n, 3, H, W, generator=g).to(torch.bfloat16).float().to(dev)
    ref = vae32.encoder.layers(img)
    x8 = torch.zeros(n * H * W, 8, dtype=torch.bfloat16, device=dev)
    x8[:, :3].copy_(to_nhwc(img).to(torch.bfloat16))
    lat = torch.zeros(n * h * w, 8, dtype=torch.bfloat16, device=dev)
    net.encode(ctx, x8, n, H, W, lat)
    torch.cuda.synchronize()
    e_enc = rel(from_nhwc(lat, n, h, w, 4), ref)
    print(f"taesd enc err {e_enc:.4f}")
    assert e_enc < 2e-2


@pytest.mark.parametrize("which,n,h,w", [("tiny", 2, 6, 8), ("sd", 1, 4, 6)])
def test_autoencoder_kl(ctx, which, n, h, w):
    """AutoencoderKL (--vae original): decoder forward + input-gradient of vae.decode(z) and the encoder's
    scaled posterior mean (prepare_latents), against the oracle's restatement of diffusers' modules
    (oracle/vae_kl_ref.py), fp32 and bf16 executions; the SD config exercises the 512-channel single-head
    mid attention."""
    from oracle.vae_kl_ref import AutoencoderKL, KLConfig, synthetic_kl_state_dict
    from depth_completion_amd.vae_kl import SD_VAE, TINY_KL, AutoencoderKLHIP
    hcfg = TINY_KL if which == "tiny" else SD_VAE
    ocfg = KLConfig(block_out_channels=hcfg.block_out_channels, layers_per_block=hcfg.layers_per_block)
    vae = AutoencoderKL(ocfg)
    sd = synthetic_kl_state_dict(vae, 21)
    vae.load_state_dict(sd)
    vae32 = vae.to(torch.bfloat16).float().to(dev)
    vae16 = AutoencoderKL(ocfg)
    vae16.load_state_dict(sd)
    vae16 = vae16.to(torch.bfloat16).to(dev)
    g = torch.Generator().manual_seed(4)
    z = torch.randn(n, 4, h, w, generator=g).to(torch.bfloat16).float().to(dev)
    zs = (z / 0.18215).to(torch.bfloat16).float().detach().requires_grad_(True)
    out = vae32.decode(zs).sample
    gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16).float().to(dev)
    out.backward(gout)
    zs16 = zs.detach().to(torch.bfloat16).requires_grad_(True)
    out16 = vae16.decode(zs16).sample
    out16.backward(gout.to(torch.bfloat16))
    e_out16, e_g16 = rel(out16, out), rel(zs16.grad, zs.grad)
    net = AutoencoderKLHIP({k: v.float() for k, v in sd.items()}, dev, hcfg)
    dp = net.decoder_plan(ctx, n, h, w)
    dp.tin.zero_()
    dp.tin[:, :4].copy_(to_nhwc(zs.detach()).to(torch.bfloat16))
    dp.forward()
    dp.dout.zero_()
    H, W = 8 * h, 8 * w
    dp.dout[:, :3].copy_(to_nhwc(2 * gout).to(torch.bfloat16))   # out holds (decoder output + 1) / 2
    dp.backward()
    torch.cuda.synchronize()
    e_out = rel(2 * from_nhwc(dp.out, n, H, W, 3) - 1, out)
    e_g = rel(from_nhwc(dp.dtin, n, h, w, 4), zs.grad)
    print(f"\nkl {which} dec out err {e_out:.4f} (oracle bf16 {e_out16:.4f}) grad err {e_g:.4f} (oracle bf16 {e_g16:.4f})")
    assert e_out <= 2 * e_out16 + 2e-3 and e_g <= 2 * e_g16 + 2e-3
    # encoder: mode() * scaling_factor of an image in [-1, 1]
    img = (torch.rand(n, 3, H, W, generator=g) * 2 - 1).to(torch.bfloat16).float().to(dev)
    ref = vae32.encode(img).latent_dist.mode() * 0.18215
    ref16 = vae16.encode(img.to(torch.bfloat16)).latent_dist.mode() * 0.18215
    x8 = torch.zeros(n * H * W, 8, dtype=torch.bfloat16, device=dev)
    x8[:, :3].copy_(to_nhwc(img).to(torch.bfloat16))
    lat = torch.zeros(n * h * w, 8, dtype=torch.bfloat16, device=dev)
    net.encode(ctx, x8, n, H, W, lat)
    torch.cuda.synchronize()
    e_enc, e_enc16 = rel(from_nhwc(lat, n, h, w, 4), ref), rel(ref16, ref)
    print(f"kl {which} enc err {e_enc:.4f} (oracle bf16 {e_enc16:.4f})")
    assert e_enc <= 2 * e_enc16 + 2e-3

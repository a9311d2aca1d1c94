"""The product's synthetic weights equal the oracle's (same keys, order, shapes, values)."""
import pytest
import torch

from depth_completion_amd import synthetic
from depth_completion_amd.config import MARIGOLD_V1, TINY
from oracle.diffusers_ref import (AutoencoderTiny, UNet2DConditionModel, UNetConfig, synthetic_state_dict,
                                  synthetic_taesd_state_dict, synthetic_text_embedding, tiny_unet_config)


@pytest.mark.parametrize("which", ["tiny", "full"])
def test_unet_synthetic_matches_oracle(which):
    m = UNet2DConditionModel(tiny_unet_config() if which == "tiny" else UNetConfig())
    shapes = synthetic.unet_shapes(TINY if which == "tiny" else MARIGOLD_V1)
    ref = m.state_dict()
    assert [k for k, _, _ in shapes] == list(ref.keys())
    assert all(tuple(ref[k].shape) == s for k, s, _ in shapes)
    if which == "tiny":
        a = synthetic.unet_state_dict(TINY, 11)
        b = synthetic_state_dict(m, 11)
        assert all(torch.equal(a[k], b[k]) for k in b)


def test_taesd_synthetic_matches_oracle():
    vae = AutoencoderTiny()
    a = synthetic.taesd_state_dict(12)
    b = synthetic_taesd_state_dict(vae, 12)
    assert list(a.keys()) == list(b.keys())
    assert all(torch.equal(a[k], b[k]) for k in b)
    assert torch.equal(synthetic.text_embedding(13, 64), synthetic_text_embedding(13, 64))


@pytest.mark.parametrize("which", ["tiny", "sd"])
def test_kl_synthetic_matches_oracle(which):
    from depth_completion_amd.vae_kl import SD_VAE, TINY_KL
    from oracle.vae_kl_ref import AutoencoderKL, KLConfig, synthetic_kl_state_dict
    hcfg = TINY_KL if which == "tiny" else SD_VAE
    vae = AutoencoderKL(KLConfig(block_out_channels=hcfg.block_out_channels, layers_per_block=hcfg.layers_per_block))
    shapes = synthetic.kl_shapes(hcfg)
    ref = vae.state_dict()
    assert [k for k, _, _ in shapes] == list(ref.keys())
    assert all(tuple(ref[k].shape) == s for k, s, _ in shapes)
    if which == "tiny":
        a = synthetic.kl_state_dict(hcfg, 7)
        b = synthetic_kl_state_dict(vae, 7)
        assert all(torch.equal(a[k], b[k]) for k in b)

"""CPU restatement of diffusers 0.31.0 ``AutoencoderKL`` (the ``--vae original`` path, predict.py:44-52).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline,
never by the product.  Follows diffusers' models/autoencoders/autoencoder_kl.py, vae.py (Encoder,
Decoder), unets/unet_2d_blocks.py (DownEncoderBlock2D, UpDecoderBlock2D, UNetMidBlock2D), resnet.py
(ResnetBlock2D without time embedding), attention_processor.py (Attention with group_norm,
residual_connection, AttnProcessor2_0 -> scaled_dot_product_attention) and the Stable Diffusion VAE
config (block_out_channels 128/256/512/512, layers_per_block 2, GroupNorm 32 eps 1e-6,
scaling_factor 0.18215).  diffusers is not installed here: the module semantics are restated from the
published library ("parity unpinned"); the reference's own use of the VAE
(prepare_latents .latent_dist.mode() * scaling_factor, decode_prediction vae.decode(z / scaling_factor))
is in oracle/pipeline_ref.py.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class KLConfig:
    block_out_channels: tuple = (128, 256, 512, 512)
    layers_per_block: int = 2
    latent_channels: int = 4
    norm_num_groups: int = 32
    scaling_factor: float = 0.18215


def tiny_kl_config() -> KLConfig:
    return KLConfig(block_out_channels=(64, 64), layers_per_block=1)


class KLResnet(nn.Module):
    """ResnetBlock2D(temb_channels=None, eps=1e-6): conv1(silu(norm1 x)) -> conv2(silu(norm2 h)) + shortcut."""

    def __init__(self, cin, cout, groups, eps=1e-6):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, cin, eps=eps)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        self.norm2 = nn.GroupNorm(groups, cout, eps=eps)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x):
        h = self.conv1(F.silu(self.norm1(x)))
        h = self.conv2(F.silu(self.norm2(h)))
        if self.conv_shortcut is not None:
            x = self.conv_shortcut(x)
        return x + h


class KLAttention(nn.Module):
    """Attention(heads=1, dim_head=C, group_norm, residual_connection=True, bias=True) via SDPA."""

    def __init__(self, c, groups, eps=1e-6):
        super().__init__()
        self.group_norm = nn.GroupNorm(groups, c, eps=eps)
        self.to_q = nn.Linear(c, c)
        self.to_k = nn.Linear(c, c)
        self.to_v = nn.Linear(c, c)
        self.to_out = nn.ModuleList([nn.Linear(c, c)])

    def forward(self, x):
        b, c, h, w = x.shape
        hs = x.view(b, c, h * w).transpose(1, 2)
        hs = self.group_norm(hs.transpose(1, 2)).transpose(1, 2)
        q, k, v = self.to_q(hs), self.to_k(hs), self.to_v(hs)
        o = F.scaled_dot_product_attention(q[:, None], k[:, None], v[:, None])[:, 0]
        o = self.to_out[0](o)
        return o.transpose(1, 2).reshape(b, c, h, w) + x


class KLMid(nn.Module):
    def __init__(self, c, groups):
        super().__init__()
        self.resnets = nn.ModuleList([KLResnet(c, c, groups), KLResnet(c, c, groups)])
        self.attentions = nn.ModuleList([KLAttention(c, groups)])

    def forward(self, x):
        x = self.resnets[0](x)
        x = self.attentions[0](x)
        return self.resnets[1](x)


class KLDownsample(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, stride=2, padding=0)

    def forward(self, x):
        return self.conv(F.pad(x, (0, 1, 0, 1)))


class KLUpsample(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, padding=1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class KLDownBlock(nn.Module):
    def __init__(self, cin, cout, n, groups, down):
        super().__init__()
        self.resnets = nn.ModuleList([KLResnet(cin if i == 0 else cout, cout, groups) for i in range(n)])
        self.downsamplers = nn.ModuleList([KLDownsample(cout)]) if down else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
        return x


class KLUpBlock(nn.Module):
    def __init__(self, cin, cout, n, groups, up):
        super().__init__()
        self.resnets = nn.ModuleList([KLResnet(cin if i == 0 else cout, cout, groups) for i in range(n)])
        self.upsamplers = nn.ModuleList([KLUpsample(cout)]) if up else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class KLEncoder(nn.Module):
    def __init__(self, cfg: KLConfig):
        super().__init__()
        ch, g = cfg.block_out_channels, cfg.norm_num_groups
        self.conv_in = nn.Conv2d(3, ch[0], 3, padding=1)
        self.down_blocks = nn.ModuleList()
        prev = ch[0]
        for i, c in enumerate(ch):
            self.down_blocks.append(KLDownBlock(prev, c, cfg.layers_per_block, g, i < len(ch) - 1))
            prev = c
        self.mid_block = KLMid(ch[-1], g)
        self.conv_norm_out = nn.GroupNorm(g, ch[-1], eps=1e-6)
        self.conv_out = nn.Conv2d(ch[-1], 2 * cfg.latent_channels, 3, padding=1)

    def forward(self, x):
        x = self.conv_in(x)
        for b in self.down_blocks:
            x = b(x)
        x = self.mid_block(x)
        return self.conv_out(F.silu(self.conv_norm_out(x)))


class KLDecoder(nn.Module):
    def __init__(self, cfg: KLConfig):
        super().__init__()
        ch, g = tuple(reversed(cfg.block_out_channels)), cfg.norm_num_groups
        self.conv_in = nn.Conv2d(cfg.latent_channels, ch[0], 3, padding=1)
        self.mid_block = KLMid(ch[0], g)
        self.up_blocks = nn.ModuleList()
        prev = ch[0]
        for i, c in enumerate(ch):
            self.up_blocks.append(KLUpBlock(prev, c, cfg.layers_per_block + 1, g, i < len(ch) - 1))
            prev = c
        self.conv_norm_out = nn.GroupNorm(g, ch[-1], eps=1e-6)
        self.conv_out = nn.Conv2d(ch[-1], 3, 3, padding=1)

    def forward(self, z):
        x = self.conv_in(z)
        x = self.mid_block(x)
        for b in self.up_blocks:
            x = b(x)
        return self.conv_out(F.silu(self.conv_norm_out(x)))


class _Dist:
    def __init__(self, moments):
        self.mean, self.logvar = torch.chunk(moments, 2, dim=1)

    def mode(self):
        return self.mean


class _Out:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class AutoencoderKL(nn.Module):
    def __init__(self, cfg: KLConfig | None = None):
        super().__init__()
        self.cfg = cfg or KLConfig()
        self.scaling_factor = self.cfg.scaling_factor
        self.encoder = KLEncoder(self.cfg)
        self.decoder = KLDecoder(self.cfg)
        lc = self.cfg.latent_channels
        self.quant_conv = nn.Conv2d(2 * lc, 2 * lc, 1)
        self.post_quant_conv = nn.Conv2d(lc, lc, 1)

    def encode(self, x, return_dict=True):
        dist = _Dist(self.quant_conv(self.encoder(x)))
        return _Out(latent_dist=dist) if return_dict else (dist,)

    def decode(self, z, return_dict=True):
        out = self.decoder(self.post_quant_conv(z))
        return _Out(sample=out) if return_dict else (out,)


def synthetic_kl_state_dict(vae: AutoencoderKL, seed: int) -> dict:
    """PyTorch-default-like seeded init (oracle.diffusers_ref.synthetic_state_dict) with a gain of 1.4 on
    the convs, so that activations keep their scale through the residual stacks."""
    from oracle.diffusers_ref import synthetic_state_dict
    return synthetic_state_dict(vae, seed, gain=1.4)

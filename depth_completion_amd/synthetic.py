"""Seeded synthetic weights in diffusers key layout (no checkpoints exist offline).

The key order, shapes and draws follow the module registration order of the restated diffusers
modules, so ``unet_state_dict(cfg, seed)`` equals the oracle's ``synthetic_state_dict`` for the
same seed (checked by tests/test_synthetic_weights.py) -- the GPU path and the CPU checker see
identical parameters.  Init: weights U(-g/sqrt(fan_in), g/sqrt(fan_in)), biases U(+-1/sqrt(fan_in))
(or +-bias_bound), norm weights 1+0.1U(-1,1), norm biases 0.1U(-1,1).
"""
from __future__ import annotations

import math

import torch

from .config import UNetConfig


def _resnet(p, cin, cout, temb):
    s = [(p + "norm1.weight", (cin,), "norm"), (p + "norm1.bias", (cin,), "norm"),
         (p + "conv1.weight", (cout, cin, 3, 3), "w"), (p + "conv1.bias", (cout,), ("b", cin * 9)),
         (p + "time_emb_proj.weight", (cout, temb), "w"), (p + "time_emb_proj.bias", (cout,), ("b", temb)),
         (p + "norm2.weight", (cout,), "norm"), (p + "norm2.bias", (cout,), "norm"),
         (p + "conv2.weight", (cout, cout, 3, 3), "w"), (p + "conv2.bias", (cout,), ("b", cout * 9))]
    if cin != cout:
        s += [(p + "conv_shortcut.weight", (cout, cin, 1, 1), "w"), (p + "conv_shortcut.bias", (cout,), ("b", cin))]
    return s


def _transformer(p, c, cross):
    b = p + "transformer_blocks.0."
    s = [(p + "norm.weight", (c,), "norm"), (p + "norm.bias", (c,), "norm"),
         (p + "proj_in.weight", (c, c), "w"), (p + "proj_in.bias", (c,), ("b", c))]
    s += [(b + "norm1.weight", (c,), "norm"), (b + "norm1.bias", (c,), "norm")]
    for a, kv in (("attn1", c), ("attn2", cross)):
        s += [(b + f"{a}.to_q.weight", (c, c), "w"), (b + f"{a}.to_k.weight", (c, kv), "w"),
              (b + f"{a}.to_v.weight", (c, kv), "w"), (b + f"{a}.to_out.0.weight", (c, c), "w"),
              (b + f"{a}.to_out.0.bias", (c,), ("b", c))]
        s += [(b + ("norm2" if a == "attn1" else "norm3") + ".weight", (c,), "norm"),
              (b + ("norm2" if a == "attn1" else "norm3") + ".bias", (c,), "norm")]
    s += [(b + "ff.net.0.proj.weight", (8 * c, c), "w"), (b + "ff.net.0.proj.bias", (8 * c,), ("b", c)),
          (b + "ff.net.2.weight", (c, 4 * c), "w"), (b + "ff.net.2.bias", (c,), ("b", 4 * c))]
    s += [(p + "proj_out.weight", (c, c), "w"), (p + "proj_out.bias", (c,), ("b", c))]
    return s


def unet_shapes(cfg: UNetConfig):
    boc = cfg.block_out_channels
    temb = cfg.time_embed_dim
    s = [("conv_in.weight", (boc[0], cfg.in_channels, 3, 3), "w"), ("conv_in.bias", (boc[0],), ("b", cfg.in_channels * 9)),
         ("time_embedding.linear_1.weight", (temb, boc[0]), "w"), ("time_embedding.linear_1.bias", (temb,), ("b", boc[0])),
         ("time_embedding.linear_2.weight", (temb, temb), "w"), ("time_embedding.linear_2.bias", (temb,), ("b", temb))]
    nb = len(boc)
    out_ch = boc[0]
    for i in range(nb):
        in_ch, out_ch = out_ch, boc[i]
        for j in range(cfg.layers_per_block):
            s += _resnet(f"down_blocks.{i}.resnets.{j}.", in_ch if j == 0 else out_ch, out_ch, temb)
        if cfg.down_attn[i]:
            for j in range(cfg.layers_per_block):
                s += _transformer(f"down_blocks.{i}.attentions.{j}.", out_ch, cfg.cross_attention_dim)
        if i < nb - 1:
            s += [(f"down_blocks.{i}.downsamplers.0.conv.weight", (out_ch, out_ch, 3, 3), "w"),
                  (f"down_blocks.{i}.downsamplers.0.conv.bias", (out_ch,), ("b", out_ch * 9))]
    c = boc[-1]
    s += _resnet("mid_block.resnets.0.", c, c, temb) + _resnet("mid_block.resnets.1.", c, c, temb)
    s += _transformer("mid_block.attentions.0.", c, cfg.cross_attention_dim)
    rev = list(reversed(boc))
    out_ch = rev[0]
    for i in range(nb):
        prev, out_ch = out_ch, rev[i]
        in_ch = rev[min(i + 1, nb - 1)]
        n_layers = cfg.layers_per_block + 1
        for j in range(n_layers):
            skip = in_ch if j == n_layers - 1 else out_ch
            rin = prev if j == 0 else out_ch
            s += _resnet(f"up_blocks.{i}.resnets.{j}.", rin + skip, out_ch, temb)
        if cfg.up_attn[i]:
            for j in range(n_layers):
                s += _transformer(f"up_blocks.{i}.attentions.{j}.", out_ch, cfg.cross_attention_dim)
        if i < nb - 1:
            s += [(f"up_blocks.{i}.upsamplers.0.conv.weight", (out_ch, out_ch, 3, 3), "w"),
                  (f"up_blocks.{i}.upsamplers.0.conv.bias", (out_ch,), ("b", out_ch * 9))]
    s += [("conv_norm_out.weight", (boc[0],), "norm"), ("conv_norm_out.bias", (boc[0],), "norm"),
          ("conv_out.weight", (cfg.out_channels, boc[0], 3, 3), "w"), ("conv_out.bias", (cfg.out_channels,), ("b", boc[0] * 9))]
    return s


def _tiny_block(p, c=64):
    s = []
    for k in (0, 2, 4):
        s += [(f"{p}conv.{k}.weight", (c, c, 3, 3), "w"), (f"{p}conv.{k}.bias", (c,), ("b", c * 9))]
    return s


def taesd_shapes():
    s = []
    i = 0
    for bi, nb in enumerate((1, 3, 3, 3)):
        if bi == 0:
            s += [(f"encoder.layers.{i}.weight", (64, 3, 3, 3), "w"), (f"encoder.layers.{i}.bias", (64,), ("b", 27))]
        else:
            s += [(f"encoder.layers.{i}.weight", (64, 64, 3, 3), "w")]
        i += 1
        for _ in range(nb):
            s += _tiny_block(f"encoder.layers.{i}.")
            i += 1
    s += [(f"encoder.layers.{i}.weight", (4, 64, 3, 3), "w"), (f"encoder.layers.{i}.bias", (4,), ("b", 576))]
    s += [("decoder.layers.0.weight", (64, 4, 3, 3), "w"), ("decoder.layers.0.bias", (64,), ("b", 36))]
    i = 2
    for bi, nb in enumerate((3, 3, 3, 1)):
        for _ in range(nb):
            s += _tiny_block(f"decoder.layers.{i}.")
            i += 1
        if bi < 3:
            i += 1
            s += [(f"decoder.layers.{i}.weight", (64, 64, 3, 3), "w")]
            i += 1
    s += [(f"decoder.layers.{i}.weight", (3, 64, 3, 3), "w"), (f"decoder.layers.{i}.bias", (3,), ("b", 576))]
    return s, i


def _fan_in(shape):
    return shape[1] * (shape[2] * shape[3] if len(shape) == 4 else 1)


def _kl_resnet(p, cin, cout):
    s = [(p + "norm1.weight", (cin,), "norm"), (p + "norm1.bias", (cin,), "norm"),
         (p + "conv1.weight", (cout, cin, 3, 3), "w"), (p + "conv1.bias", (cout,), ("b", cin * 9)),
         (p + "norm2.weight", (cout,), "norm"), (p + "norm2.bias", (cout,), "norm"),
         (p + "conv2.weight", (cout, cout, 3, 3), "w"), (p + "conv2.bias", (cout,), ("b", cout * 9))]
    if cin != cout:
        s += [(p + "conv_shortcut.weight", (cout, cin, 1, 1), "w"), (p + "conv_shortcut.bias", (cout,), ("b", cin))]
    return s


def _kl_mid(p, c):
    s = _kl_resnet(p + "resnets.0.", c, c) + _kl_resnet(p + "resnets.1.", c, c)
    a = p + "attentions.0."
    s += [(a + "group_norm.weight", (c,), "norm"), (a + "group_norm.bias", (c,), "norm")]
    for n in ("to_q", "to_k", "to_v", "to_out.0"):
        s += [(a + n + ".weight", (c, c), "w"), (a + n + ".bias", (c,), ("b", c))]
    return s


def kl_shapes(cfg):
    """AutoencoderKL (diffusers key layout) in the oracle module's registration order."""
    ch, L, lc = cfg.block_out_channels, cfg.layers_per_block, cfg.latent_channels
    s = [("encoder.conv_in.weight", (ch[0], 3, 3, 3), "w"), ("encoder.conv_in.bias", (ch[0],), ("b", 27))]
    prev = ch[0]
    for i, c in enumerate(ch):
        for j in range(L):
            s += _kl_resnet(f"encoder.down_blocks.{i}.resnets.{j}.", prev if j == 0 else c, c)
        if i < len(ch) - 1:
            p = f"encoder.down_blocks.{i}.downsamplers.0.conv."
            s += [(p + "weight", (c, c, 3, 3), "w"), (p + "bias", (c,), ("b", c * 9))]
        prev = c
    s += _kl_mid("encoder.mid_block.", ch[-1])
    s += [("encoder.conv_norm_out.weight", (ch[-1],), "norm"), ("encoder.conv_norm_out.bias", (ch[-1],), "norm"),
          ("encoder.conv_out.weight", (2 * lc, ch[-1], 3, 3), "w"), ("encoder.conv_out.bias", (2 * lc,), ("b", ch[-1] * 9))]
    rch = tuple(reversed(ch))
    s += [("decoder.conv_in.weight", (rch[0], lc, 3, 3), "w"), ("decoder.conv_in.bias", (rch[0],), ("b", lc * 9))]
    s += _kl_mid("decoder.mid_block.", rch[0])
    prev = rch[0]
    for i, c in enumerate(rch):
        for j in range(L + 1):
            s += _kl_resnet(f"decoder.up_blocks.{i}.resnets.{j}.", prev if j == 0 else c, c)
        if i < len(rch) - 1:
            p = f"decoder.up_blocks.{i}.upsamplers.0.conv."
            s += [(p + "weight", (c, c, 3, 3), "w"), (p + "bias", (c,), ("b", c * 9))]
        prev = c
    s += [("decoder.conv_norm_out.weight", (rch[-1],), "norm"), ("decoder.conv_norm_out.bias", (rch[-1],), "norm"),
          ("decoder.conv_out.weight", (3, rch[-1], 3, 3), "w"), ("decoder.conv_out.bias", (3,), ("b", rch[-1] * 9))]
    s += [("quant_conv.weight", (2 * lc, 2 * lc, 1, 1), "w"), ("quant_conv.bias", (2 * lc,), ("b", 2 * lc)),
          ("post_quant_conv.weight", (lc, lc, 1, 1), "w"), ("post_quant_conv.bias", (lc,), ("b", lc))]
    return s


def generate(shapes, seed: int, gain: float = 1.0, bias_bound: float | None = None) -> dict:
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, shape, kind in shapes:
        if kind == "norm":
            u = torch.rand(shape, generator=g) * 2 - 1
            sd[name] = (1.0 + 0.1 * u) if name.endswith("weight") else 0.1 * u
        elif kind == "w":
            sd[name] = (torch.rand(shape, generator=g) * 2 - 1) * (gain / math.sqrt(_fan_in(shape)))
        else:
            bound = bias_bound if bias_bound is not None else 1.0 / math.sqrt(kind[1])
            sd[name] = (torch.rand(shape, generator=g) * 2 - 1) * bound
    return sd


def unet_state_dict(cfg: UNetConfig, seed: int = 11) -> dict:
    return generate(unet_shapes(cfg), seed)


def taesd_state_dict(seed: int = 12) -> dict:
    shapes, last = taesd_shapes()
    sd = generate(shapes, seed, gain=1.6, bias_bound=0.1)
    sd[f"decoder.layers.{last}.bias"] = sd[f"decoder.layers.{last}.bias"] + 0.5
    return sd


def text_embedding(seed: int = 13, cross_dim: int = 1024) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randn((1, 2, cross_dim), generator=g)


def kl_state_dict(cfg, seed: int = 12) -> dict:
    """AutoencoderKL weights; equal to oracle.vae_kl_ref.synthetic_kl_state_dict for the same seed."""
    return generate(kl_shapes(cfg), seed, gain=1.4)

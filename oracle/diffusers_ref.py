"""CPU restatement of the diffusers 0.31.0 components on the Marigold-DC hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``depth_completion_amd`` may import this
module: it is the checker for the HIP path (``tests/``, ``__graft_entry__.smoke``
and ``bench.py``'s ``cpu_baseline`` leg only).

The reference (``/root/reference/marigold_dc.py``) calls into diffusers 0.31.0
(``requirements.txt:1``), which is not installed in this image.  The modules
below restate the published semantics of the classes the reference uses, with
the same attribute hierarchy so that a diffusers-format state dict loads 1:1:

* ``UNet2DConditionModel`` (SD2 architecture, Marigold v1-0: 8 input channels)
  -- used by ``_predict_noise`` (marigold_dc.py:432-465)
* ``AutoencoderTiny`` (TAESD) -- swapped in by predict.py:484-488, used by
  ``prepare_latents`` (marigold_dc.py:696-698) and ``decode_prediction``
  (marigold_dc.py:366)
* ``DDIMScheduler`` with ``timestep_spacing="trailing"`` (predict.py:491-494),
  used at marigold_dc.py:800, 814, 823-826, 902-909
* ``MarigoldImageProcessor`` (preprocess/unpad/resize, marigold_dc.py:367-370,
  687-692)

Parity status of this file: the diffusers source is absent, so the
restatement follows SURVEY.md Appendix A; module semantics are "parity
unpinned" against diffusers itself.  The reference's own guidance code
(marigold_dc.py / utils.py) is pinned separately by golden vectors produced
by running that code (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------
# UNet2DConditionModel (diffusers/models/unets/unet_2d_condition.py)
# --------------------------------------------------------------------------
@dataclass
class UNetConfig:
    """Marigold v1-0 UNet config (SD2 architecture).  SURVEY.md Appendix A."""

    in_channels: int = 8
    out_channels: int = 4
    block_out_channels: tuple = (320, 640, 1280, 1280)
    layers_per_block: int = 2
    heads: tuple = (5, 10, 20, 20)  # diffusers' "attention_head_dim" (head dim 64)
    cross_attention_dim: int = 1024
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    # down: 3x CrossAttnDownBlock2D + DownBlock2D ; up: UpBlock2D + 3x CrossAttnUpBlock2D
    down_attn: tuple = (True, True, True, False)
    up_attn: tuple = (False, True, True, True)

    @property
    def time_embed_dim(self) -> int:
        return self.block_out_channels[0] * 4


def tiny_unet_config() -> UNetConfig:
    """Reduced-width config with the same topology (tests / golden vectors)."""
    return UNetConfig(
        block_out_channels=(64, 128, 128, 128),
        heads=(1, 2, 2, 2),
        cross_attention_dim=64,
    )


def get_timestep_embedding(timesteps, embedding_dim, flip_sin_to_cos=False,
                           downscale_freq_shift=1.0, scale=1.0, max_period=10000):
    half_dim = embedding_dim // 2
    exponent = -math.log(max_period) * torch.arange(
        start=0, end=half_dim, dtype=torch.float32, device=timesteps.device)
    exponent = exponent / (half_dim - downscale_freq_shift)
    emb = torch.exp(exponent)
    emb = timesteps[:, None].float() * emb[None, :]
    emb = scale * emb
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half_dim:], emb[:, :half_dim]], dim=-1)
    if embedding_dim % 2 == 1:
        emb = F.pad(emb, (0, 1, 0, 0))
    return emb


class Timesteps(nn.Module):
    def __init__(self, num_channels, flip_sin_to_cos, downscale_freq_shift):
        super().__init__()
        self.num_channels = num_channels
        self.flip_sin_to_cos = flip_sin_to_cos
        self.downscale_freq_shift = downscale_freq_shift

    def forward(self, timesteps):
        return get_timestep_embedding(timesteps, self.num_channels,
                                      flip_sin_to_cos=self.flip_sin_to_cos,
                                      downscale_freq_shift=self.downscale_freq_shift)


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels, time_embed_dim):
        super().__init__()
        self.linear_1 = nn.Linear(in_channels, time_embed_dim)
        self.act = nn.SiLU()
        self.linear_2 = nn.Linear(time_embed_dim, time_embed_dim)

    def forward(self, sample):
        return self.linear_2(self.act(self.linear_1(sample)))


class ResnetBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, groups=32, eps=1e-5):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, 1, 1)
        self.time_emb_proj = nn.Linear(temb_channels, out_channels)
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, 1, 1)
        self.nonlinearity = nn.SiLU()
        self.use_in_shortcut = in_channels != out_channels
        self.conv_shortcut = (nn.Conv2d(in_channels, out_channels, 1, 1, 0)
                              if self.use_in_shortcut else None)
        self.output_scale_factor = 1.0

    def forward(self, input_tensor, temb):
        hidden_states = input_tensor
        hidden_states = self.norm1(hidden_states)
        hidden_states = self.nonlinearity(hidden_states)
        hidden_states = self.conv1(hidden_states)
        temb = self.nonlinearity(temb)
        temb = self.time_emb_proj(temb)[:, :, None, None]
        hidden_states = hidden_states + temb
        hidden_states = self.norm2(hidden_states)
        hidden_states = self.nonlinearity(hidden_states)
        hidden_states = self.dropout(hidden_states)
        hidden_states = self.conv2(hidden_states)
        if self.conv_shortcut is not None:
            input_tensor = self.conv_shortcut(input_tensor)
        return (input_tensor + hidden_states) / self.output_scale_factor


class Attention(nn.Module):
    """AttnProcessor2_0 semantics: SDPA, q/k/v without bias, out with bias."""

    def __init__(self, query_dim, cross_attention_dim=None, heads=8, dim_head=64):
        super().__init__()
        inner = heads * dim_head
        self.heads = heads
        kv_dim = cross_attention_dim if cross_attention_dim is not None else query_dim
        self.to_q = nn.Linear(query_dim, inner, bias=False)
        self.to_k = nn.Linear(kv_dim, inner, bias=False)
        self.to_v = nn.Linear(kv_dim, inner, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim, bias=True), nn.Dropout(0.0)])
        self.rescale_output_factor = 1.0

    def forward(self, hidden_states, encoder_hidden_states=None):
        b, _, _ = hidden_states.shape
        if encoder_hidden_states is None:
            encoder_hidden_states = hidden_states
        q = self.to_q(hidden_states)
        k = self.to_k(encoder_hidden_states)
        v = self.to_v(encoder_hidden_states)
        inner = k.shape[-1]
        hd = inner // self.heads
        q = q.view(b, -1, self.heads, hd).transpose(1, 2)
        k = k.view(b, -1, self.heads, hd).transpose(1, 2)
        v = v.view(b, -1, self.heads, hd).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=0.0, is_causal=False)
        o = o.transpose(1, 2).reshape(b, -1, self.heads * hd).to(q.dtype)
        o = self.to_out[0](o)
        o = self.to_out[1](o)
        return o / self.rescale_output_factor


class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2, bias=True)

    def forward(self, hidden_states):
        hidden_states = self.proj(hidden_states)
        hidden_states, gate = hidden_states.chunk(2, dim=-1)
        return hidden_states * F.gelu(gate)


class FeedForward(nn.Module):
    def __init__(self, dim, mult=4):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([GEGLU(dim, inner), nn.Dropout(0.0), nn.Linear(inner, dim, bias=True)])

    def forward(self, hidden_states):
        for m in self.net:
            hidden_states = m(hidden_states)
        return hidden_states


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, heads, dim_head, cross_attention_dim):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, elementwise_affine=True, eps=1e-5)
        self.attn1 = Attention(dim, None, heads, dim_head)
        self.norm2 = nn.LayerNorm(dim, elementwise_affine=True, eps=1e-5)
        self.attn2 = Attention(dim, cross_attention_dim, heads, dim_head)
        self.norm3 = nn.LayerNorm(dim, elementwise_affine=True, eps=1e-5)
        self.ff = FeedForward(dim)

    def forward(self, hidden_states, encoder_hidden_states):
        n = self.norm1(hidden_states)
        hidden_states = self.attn1(n) + hidden_states
        n = self.norm2(hidden_states)
        hidden_states = self.attn2(n, encoder_hidden_states) + hidden_states
        n = self.norm3(hidden_states)
        hidden_states = self.ff(n) + hidden_states
        return hidden_states


class Transformer2DModel(nn.Module):
    """use_linear_projection=True (SD2)."""

    def __init__(self, heads, dim_head, in_channels, cross_attention_dim, groups=32):
        super().__init__()
        inner = heads * dim_head
        self.norm = nn.GroupNorm(groups, in_channels, eps=1e-6, affine=True)
        self.proj_in = nn.Linear(in_channels, inner)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(inner, heads, dim_head, cross_attention_dim)])
        self.proj_out = nn.Linear(inner, in_channels)

    def forward(self, hidden_states, encoder_hidden_states):
        b, c, h, w = hidden_states.shape
        residual = hidden_states
        hidden_states = self.norm(hidden_states)
        inner = hidden_states.shape[1]
        hidden_states = hidden_states.permute(0, 2, 3, 1).reshape(b, h * w, inner)
        hidden_states = self.proj_in(hidden_states)
        for blk in self.transformer_blocks:
            hidden_states = blk(hidden_states, encoder_hidden_states)
        hidden_states = self.proj_out(hidden_states)
        hidden_states = hidden_states.reshape(b, h, w, inner).permute(0, 3, 1, 2).contiguous()
        return hidden_states + residual


class Downsample2D(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=1)

    def forward(self, x):
        return self.conv(x)


class Upsample2D(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, padding=1)

    def forward(self, x, output_size=None):
        dtype = x.dtype
        if dtype == torch.bfloat16:
            x = x.to(torch.float32)
        if output_size is None:
            x = F.interpolate(x, scale_factor=2.0, mode="nearest")
        else:
            x = F.interpolate(x, size=output_size, mode="nearest")
        if dtype == torch.bfloat16:
            x = x.to(dtype)
        return self.conv(x)


class DownBlock(nn.Module):
    """CrossAttnDownBlock2D (with attentions) or DownBlock2D."""

    def __init__(self, in_ch, out_ch, temb, n_layers, heads, cross_dim, with_attn, add_down, groups):
        super().__init__()
        self.resnets = nn.ModuleList([
            ResnetBlock2D(in_ch if i == 0 else out_ch, out_ch, temb, groups) for i in range(n_layers)])
        if with_attn:
            self.attentions = nn.ModuleList([
                Transformer2DModel(heads, out_ch // heads, out_ch, cross_dim, groups) for _ in range(n_layers)])
        else:
            self.attentions = None
        self.downsamplers = nn.ModuleList([Downsample2D(out_ch)]) if add_down else None

    def forward(self, h, temb, ctx):
        outs = ()
        for i, r in enumerate(self.resnets):
            h = r(h, temb)
            if self.attentions is not None:
                h = self.attentions[i](h, ctx)
            outs = outs + (h,)
        if self.downsamplers is not None:
            for d in self.downsamplers:
                h = d(h)
            outs = outs + (h,)
        return h, outs


class UpBlock(nn.Module):
    """UpBlock2D (no attentions) or CrossAttnUpBlock2D."""

    def __init__(self, in_ch, out_ch, prev_out_ch, temb, n_layers, heads, cross_dim, with_attn, add_up, groups):
        super().__init__()
        res = []
        for i in range(n_layers):
            res_skip = in_ch if i == n_layers - 1 else out_ch
            res_in = prev_out_ch if i == 0 else out_ch
            res.append(ResnetBlock2D(res_in + res_skip, out_ch, temb, groups))
        self.resnets = nn.ModuleList(res)
        if with_attn:
            self.attentions = nn.ModuleList([
                Transformer2DModel(heads, out_ch // heads, out_ch, cross_dim, groups) for _ in range(n_layers)])
        else:
            self.attentions = None
        self.upsamplers = nn.ModuleList([Upsample2D(out_ch)]) if add_up else None

    def forward(self, h, res_samples, temb, ctx, upsample_size=None):
        for i, r in enumerate(self.resnets):
            skip = res_samples[-1]
            res_samples = res_samples[:-1]
            h = torch.cat([h, skip], dim=1)
            h = r(h, temb)
            if self.attentions is not None:
                h = self.attentions[i](h, ctx)
        if self.upsamplers is not None:
            for u in self.upsamplers:
                h = u(h, upsample_size)
        return h


class MidBlock(nn.Module):
    def __init__(self, ch, temb, heads, cross_dim, groups):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, temb, groups), ResnetBlock2D(ch, ch, temb, groups)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, ch // heads, ch, cross_dim, groups)])

    def forward(self, h, temb, ctx):
        h = self.resnets[0](h, temb)
        h = self.attentions[0](h, ctx)
        h = self.resnets[1](h, temb)
        return h


class UNet2DConditionModel(nn.Module):
    def __init__(self, cfg: UNetConfig | None = None):
        super().__init__()
        cfg = cfg or UNetConfig()
        self.config = cfg
        boc = cfg.block_out_channels
        g = cfg.norm_num_groups
        temb = cfg.time_embed_dim
        self.conv_in = nn.Conv2d(cfg.in_channels, boc[0], 3, padding=1)
        self.time_proj = Timesteps(boc[0], True, 0)
        self.time_embedding = TimestepEmbedding(boc[0], temb)
        self.down_blocks = nn.ModuleList()
        out_ch = boc[0]
        nb = len(boc)
        for i in range(nb):
            in_ch, out_ch = out_ch, boc[i]
            self.down_blocks.append(DownBlock(in_ch, out_ch, temb, cfg.layers_per_block, cfg.heads[i],
                                              cfg.cross_attention_dim, cfg.down_attn[i], i < nb - 1, g))
        self.mid_block = MidBlock(boc[-1], temb, cfg.heads[-1], cfg.cross_attention_dim, g)
        rev = list(reversed(boc))
        rev_heads = list(reversed(cfg.heads))
        self.up_blocks = nn.ModuleList()
        out_ch = rev[0]
        for i in range(nb):
            prev = out_ch
            out_ch = rev[i]
            in_ch = rev[min(i + 1, nb - 1)]
            self.up_blocks.append(UpBlock(in_ch, out_ch, prev, temb, cfg.layers_per_block + 1, rev_heads[i],
                                          cfg.cross_attention_dim, cfg.up_attn[i], i < nb - 1, g))
        self.conv_norm_out = nn.GroupNorm(g, boc[0], eps=cfg.norm_eps)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(boc[0], cfg.out_channels, 3, padding=1)

    @property
    def num_upsamplers(self):
        return len(self.config.block_out_channels) - 1

    def forward(self, sample, timestep, encoder_hidden_states, return_dict=False):
        up_factor = 2 ** self.num_upsamplers
        forward_upsample_size = any(s % up_factor != 0 for s in sample.shape[-2:])
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], dtype=torch.int64, device=sample.device)
        elif timestep.ndim == 0:
            timestep = timestep[None].to(sample.device)
        timesteps = timestep.expand(sample.shape[0])
        t_emb = self.time_proj(timesteps).to(dtype=sample.dtype)
        emb = self.time_embedding(t_emb)
        h = self.conv_in(sample)
        res = (h,)
        for blk in self.down_blocks:
            h, r = blk(h, emb, encoder_hidden_states)
            res = res + r
        h = self.mid_block(h, emb, encoder_hidden_states)
        for i, blk in enumerate(self.up_blocks):
            is_final = i == len(self.up_blocks) - 1
            n = len(blk.resnets)
            rs = res[-n:]
            res = res[:-n]
            upsample_size = res[-1].shape[2:] if (not is_final and forward_upsample_size) else None
            h = blk(h, rs, emb, encoder_hidden_states, upsample_size)
        h = self.conv_norm_out(h)
        h = self.conv_act(h)
        h = self.conv_out(h)
        return (h,)


# --------------------------------------------------------------------------
# AutoencoderTiny (TAESD; diffusers/models/autoencoders/autoencoder_tiny.py + vae.py)
# --------------------------------------------------------------------------
class AutoencoderTinyBlock(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, 3, padding=1), nn.ReLU(),
            nn.Conv2d(out_channels, out_channels, 3, padding=1), nn.ReLU(),
            nn.Conv2d(out_channels, out_channels, 3, padding=1))
        self.skip = (nn.Conv2d(in_channels, out_channels, 1, bias=False)
                     if in_channels != out_channels else nn.Identity())
        self.fuse = nn.ReLU()

    def forward(self, x):
        return self.fuse(self.conv(x) + self.skip(x))


class EncoderTiny(nn.Module):
    def __init__(self, in_channels=3, out_channels=4, num_blocks=(1, 3, 3, 3), ch=(64, 64, 64, 64)):
        super().__init__()
        layers = []
        for i, nb in enumerate(num_blocks):
            c = ch[i]
            if i == 0:
                layers.append(nn.Conv2d(in_channels, c, 3, padding=1))
            else:
                layers.append(nn.Conv2d(c, c, 3, padding=1, stride=2, bias=False))
            for _ in range(nb):
                layers.append(AutoencoderTinyBlock(c, c))
        layers.append(nn.Conv2d(ch[-1], out_channels, 3, padding=1))
        self.layers = nn.Sequential(*layers)

    def forward(self, x):
        # scale image from [-1, 1] to [0, 1] to match TAESD convention
        return self.layers(x.add(1).div(2))


class DecoderTiny(nn.Module):
    def __init__(self, in_channels=4, out_channels=3, num_blocks=(3, 3, 3, 1), ch=(64, 64, 64, 64)):
        super().__init__()
        layers = [nn.Conv2d(in_channels, ch[0], 3, padding=1), nn.ReLU()]
        for i, nb in enumerate(num_blocks):
            final = i == len(num_blocks) - 1
            c = ch[i]
            for _ in range(nb):
                layers.append(AutoencoderTinyBlock(c, c))
            if not final:
                layers.append(nn.Upsample(scale_factor=2, mode="nearest"))
            layers.append(nn.Conv2d(c, c if not final else out_channels, 3, padding=1, bias=final))
        self.layers = nn.Sequential(*layers)

    def forward(self, x):
        x = torch.tanh(x / 3) * 3
        x = self.layers(x)
        # scale image from [0, 1] to [-1, 1] to match diffusers convention
        return x.mul(2).sub(1)


class _Out:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class AutoencoderTiny(nn.Module):
    scaling_factor = 1.0
    latent_channels = 4

    def __init__(self):
        super().__init__()
        self.encoder = EncoderTiny()
        self.decoder = DecoderTiny()

    def encode(self, x, return_dict=True):
        out = self.encoder(x)
        return _Out(latents=out) if return_dict else (out,)

    def decode(self, x, return_dict=True):
        out = self.decoder(x)
        return _Out(sample=out) if return_dict else (out,)


# --------------------------------------------------------------------------
# DDIMScheduler (diffusers/schedulers/scheduling_ddim.py), Marigold v1-0 config
# --------------------------------------------------------------------------
@dataclass
class DDIMConfig:
    num_train_timesteps: int = 1000
    beta_start: float = 0.00085
    beta_end: float = 0.012
    beta_schedule: str = "scaled_linear"
    prediction_type: str = "v_prediction"
    set_alpha_to_one: bool = False
    steps_offset: int = 1
    timestep_spacing: str = "trailing"   # forced by predict.py:491-494
    clip_sample: bool = False


class DDIMScheduler:
    def __init__(self, config: DDIMConfig | None = None):
        self.config = config or DDIMConfig()
        c = self.config
        assert c.beta_schedule == "scaled_linear"
        self.betas = torch.linspace(c.beta_start ** 0.5, c.beta_end ** 0.5, c.num_train_timesteps,
                                    dtype=torch.float32) ** 2
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if c.set_alpha_to_one else self.alphas_cumprod[0]
        self.num_inference_steps = None
        self.timesteps = None

    def set_timesteps(self, num_inference_steps, device=None):
        import numpy as np
        c = self.config
        self.num_inference_steps = num_inference_steps
        if c.timestep_spacing == "trailing":
            step_ratio = c.num_train_timesteps / num_inference_steps
            ts = np.round(np.arange(c.num_train_timesteps, 0, -step_ratio)).astype(np.int64)
            ts -= 1
        elif c.timestep_spacing == "leading":
            step_ratio = c.num_train_timesteps // num_inference_steps
            ts = (np.arange(0, num_inference_steps) * step_ratio).round()[::-1].copy().astype(np.int64)
            ts += c.steps_offset
        else:
            raise ValueError(c.timestep_spacing)
        self.timesteps = torch.from_numpy(ts).to(device)

    def step(self, model_output, timestep, sample, eta=0.0, generator=None, return_dict=True):
        c = self.config
        prev_timestep = timestep - c.num_train_timesteps // self.num_inference_steps
        alpha_prod_t = self.alphas_cumprod[timestep]
        alpha_prod_t_prev = (self.alphas_cumprod[prev_timestep] if prev_timestep >= 0
                             else self.final_alpha_cumprod)
        beta_prod_t = 1 - alpha_prod_t
        if c.prediction_type == "v_prediction":
            pred_original_sample = (alpha_prod_t ** 0.5) * sample - (beta_prod_t ** 0.5) * model_output
            pred_epsilon = (alpha_prod_t ** 0.5) * model_output + (beta_prod_t ** 0.5) * sample
        elif c.prediction_type == "epsilon":
            pred_original_sample = (sample - beta_prod_t ** 0.5 * model_output) / alpha_prod_t ** 0.5
            pred_epsilon = model_output
        else:
            raise ValueError(c.prediction_type)
        beta_prod_t_prev = 1 - alpha_prod_t_prev
        variance = (beta_prod_t_prev / beta_prod_t) * (1 - alpha_prod_t / alpha_prod_t_prev)
        std_dev_t = eta * variance ** 0.5
        pred_sample_direction = (1 - alpha_prod_t_prev - std_dev_t ** 2) ** 0.5 * pred_epsilon
        prev_sample = alpha_prod_t_prev ** 0.5 * pred_original_sample + pred_sample_direction
        return _Out(prev_sample=prev_sample, pred_original_sample=pred_original_sample)


# --------------------------------------------------------------------------
# MarigoldImageProcessor (diffusers/pipelines/marigold/marigold_image_processing.py)
# --------------------------------------------------------------------------
class MarigoldImageProcessor:
    vae_scale_factor = 8

    @staticmethod
    def load_image_canonical(image, device, dtype):
        if image.ndim == 3:
            image = image[None]
        dmax = None
        if not torch.is_floating_point(image):
            if image.dtype != torch.uint8:
                raise ValueError(f"Image dtype={image.dtype} is not supported.")
            dmax = 255
        if image.shape[1] == 1:
            image = image.repeat(1, 3, 1, 1)
        if image.shape[1] != 3:
            raise ValueError("Input image is not 1- or 3-channel")
        image = image.to(device=device, dtype=dtype)
        if dmax is not None:
            image = image / dmax
        return image

    @staticmethod
    def resize_antialias(image, size, mode, is_aa=None):
        antialias = bool(is_aa) and mode in ("bilinear", "bicubic")
        if antialias and image.dtype == torch.bfloat16 and image.device.type == "cpu":
            # PyTorch's CPU backend has no bf16 antialiased resize: the CPU bf16 oracle (the tests' deterministic
            # anchor) resizes in fp32 and rounds the result to bf16 -- a deviation of that leg only, never of the
            # fp32 leg, and only where the bf16 call would raise
            return F.interpolate(image.float(), size, mode=mode, antialias=True).to(torch.bfloat16)
        return F.interpolate(image, size, mode=mode, antialias=antialias)

    @staticmethod
    def resize_to_max_edge(image, max_edge_sz, mode):
        h, w = image.shape[-2:]
        max_orig = max(h, w)
        new_h = h * max_edge_sz // max_orig
        new_w = w * max_edge_sz // max_orig
        if new_h == 0 or new_w == 0:
            raise ValueError(f"Extreme aspect ratio of the input image: [{w} x {h}]")
        return MarigoldImageProcessor.resize_antialias(image, (new_h, new_w), mode, is_aa=True)

    @staticmethod
    def pad_image(image, align):
        h, w = image.shape[-2:]
        ph, pw = -h % align, -w % align
        image = F.pad(image, (0, pw, 0, ph), mode="replicate")
        return image, (ph, pw)

    @staticmethod
    def unpad_image(image, padding):
        ph, pw = padding
        uh = None if ph == 0 else -ph
        uw = None if pw == 0 else -pw
        return image[:, :, :uh, :uw]

    def preprocess(self, image, processing_resolution=None, resample_method_input="bilinear",
                   device="cpu", dtype=torch.float32):
        image = self.load_image_canonical(image, device, dtype)
        original_resolution = image.shape[2:]
        image = image * 2.0 - 1.0
        if processing_resolution is not None and processing_resolution > 0:
            image = self.resize_to_max_edge(image, processing_resolution, resample_method_input)
        image, padding = self.pad_image(image, self.vae_scale_factor)
        return image, padding, original_resolution


# --------------------------------------------------------------------------
# Synthetic, seeded weights (no checkpoints are available offline)
# --------------------------------------------------------------------------
def synthetic_state_dict(module: nn.Module, seed: int, gain: float = 1.0, bias_bound: float | None = None) -> dict:
    """Deterministic PyTorch-default-like init, generated on the CPU from ``seed``.

    Linear/Conv weights ~ U(-g/sqrt(fan_in), g/sqrt(fan_in)) (g=1 is kaiming_uniform a=sqrt(5));
    biases ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)) or U(-bias_bound, bias_bound); norm weights
    1 + 0.1*U(-1,1), norm biases 0.1*U(-1,1) (non-trivial so that affine paths are exercised).
    """
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, p in module.state_dict().items():
        shape = p.shape
        parts = name.split(".")
        owner = module
        for q in parts[:-1]:
            owner = getattr(owner, q) if not q.isdigit() else owner[int(q)]
        if isinstance(owner, (nn.GroupNorm, nn.LayerNorm)):
            u = torch.rand(shape, generator=g) * 2 - 1
            sd[name] = (1.0 + 0.1 * u) if parts[-1] == "weight" else 0.1 * u
        else:
            if isinstance(owner, nn.Conv2d):
                fan_in = owner.in_channels * owner.kernel_size[0] * owner.kernel_size[1]
            elif isinstance(owner, nn.Linear):
                fan_in = owner.in_features
            else:
                raise TypeError(f"unexpected parameter owner for {name}: {type(owner)}")
            if parts[-1] == "weight":
                bound = gain / math.sqrt(fan_in)
            else:
                bound = bias_bound if bias_bound is not None else 1.0 / math.sqrt(fan_in)
            sd[name] = (torch.rand(shape, generator=g) * 2 - 1) * bound
    return sd


def synthetic_taesd_state_dict(vae: nn.Module, seed: int) -> dict:
    """TAESD init with a ReLU gain (1.6) and a decoder output bias of 0.5, so that synthetic
    decodes land inside the clip range of ``decode_prediction`` (gradients flow)."""
    sd = synthetic_state_dict(vae, seed, gain=1.6, bias_bound=0.1)
    last = len(vae.decoder.layers) - 1
    sd[f"decoder.layers.{last}.bias"] = sd[f"decoder.layers.{last}.bias"] + 0.5
    return sd


def synthetic_text_embedding(seed: int, cross_dim: int) -> torch.Tensor:
    """Stand-in for the empty-prompt CLIP embedding (marigold_dc.py:663-674): [1, 2, cross_dim]."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn((1, 2, cross_dim), generator=g)


__all__ = [
    "UNetConfig", "tiny_unet_config", "UNet2DConditionModel", "AutoencoderTiny", "DDIMScheduler",
    "DDIMConfig", "MarigoldImageProcessor", "synthetic_state_dict", "synthetic_taesd_state_dict",
    "synthetic_text_embedding",
]

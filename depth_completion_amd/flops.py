"""Algorithmic FLOPs of the guided sampler (SURVEY.md §8d convention), for the frame roofline.

Counts the reference algorithm's work -- not what this build executes (the sparse-aware decode and the
folded cross-attention do less) -- so the fraction of peak is comparable across builds:
  * 2 * M * N * K per conv / linear (all 9 taps; stride-2 convs over their output pixels);
  * attention QK^T + PV = 4 * T^2 * C per self-attention, and the same over the 2 context tokens for
    the cross-attention; its projections (q, out) as linears;
  * input-gradient = forward for every conv / linear (conv_in: only the 4 depth-latent channels);
    attention backward = 2x its forward matmuls (no recompute); no weight-gradients;
  * per guided step: UNet fwd + dgrad, TAESD decoder fwd + dgrad; once per frame: TAESD encoder and one
    final decoder forward.
Reproduces SURVEY §8d's table (C2: 190.4 TFLOP / frame; tests/test_flops.py).
"""
from __future__ import annotations

from .config import MARIGOLD_V1, UNetConfig


def _conv(p, cin, cout, k=3):
    return 2.0 * p * cout * cin * k * k


def unet_flops(h: int, w: int, cfg: UNetConfig = MARIGOLD_V1, ctx_tokens: int = 2, ctx_dim: int = 1024):
    """(forward, input-gradient) FLOPs of one UNet evaluation of one frame at latent h x w."""
    boc = cfg.block_out_channels
    nlev = len(boc)
    sizes = [(h, w)]
    for _ in range(nlev - 1):
        hh, ww = sizes[-1]
        sizes.append(((hh - 1) // 2 + 1, (ww - 1) // 2 + 1))
    px = [a * b for a, b in sizes]
    fwd = 0.0
    bwd = 0.0

    def lin(p, cin, cout):
        return 2.0 * p * cin * cout

    def resnet(p, cin, cout):
        f = _conv(p, cin, cout) + _conv(p, cout, cout)
        if cin != cout:
            f += _conv(p, cin, cout, 1)
        return f

    def transformer(p, c):
        proj = lin(p, c, c) * 2                       # proj_in, proj_out
        self_lin = lin(p, c, 3 * c) + lin(p, c, c)    # q, k, v, out
        self_att = 4.0 * p * p * c
        cross_lin = lin(p, c, c) * 2 + 2 * lin(ctx_tokens, ctx_dim, c)   # q, out; k, v of the context
        cross_att = 4.0 * p * ctx_tokens * c
        ff = lin(p, c, 8 * c) + lin(p, 4 * c, c)
        lin_total = proj + self_lin + cross_lin + ff
        att = self_att + cross_att
        return lin_total + att, lin_total + 2 * att   # (forward, input-gradient)

    # conv_in (8 -> C0): input-gradient for the 4 depth-latent channels only
    fwd += _conv(px[0], cfg.in_channels, boc[0])
    bwd += _conv(px[0], cfg.in_channels // 2, boc[0])
    skips = [boc[0]]
    ch = boc[0]
    for i in range(nlev):
        for _ in range(cfg.layers_per_block):
            f = resnet(px[i], ch, boc[i])
            fwd += f
            bwd += f
            ch = boc[i]
            if cfg.down_attn[i]:
                f, b = transformer(px[i], ch)
                fwd += f
                bwd += b
            skips.append(ch)
        if i < nlev - 1:
            f = _conv(px[i + 1], ch, ch)
            fwd += f
            bwd += f
            skips.append(ch)
    for k in range(2):   # mid block: resnet, transformer, resnet
        f = resnet(px[-1], ch, ch)
        fwd += f
        bwd += f
        if k == 0:
            f, b = transformer(px[-1], ch)
            fwd += f
            bwd += b
    rev = list(reversed(boc))
    for i in range(nlev):
        lev = nlev - 1 - i
        for _ in range(cfg.layers_per_block + 1):
            s = skips.pop()
            f = resnet(px[lev], ch + s, rev[i])
            fwd += f
            bwd += f
            ch = rev[i]
            if cfg.up_attn[i]:
                f, b = transformer(px[lev], ch)
                fwd += f
                bwd += b
        if i < nlev - 1:
            f = _conv(px[lev - 1], ch, ch)   # nearest upsample then conv at the next level's size
            fwd += f
            bwd += f
    f = _conv(px[0], boc[0], cfg.out_channels)
    fwd += f
    bwd += f
    return fwd, bwd


def taesd_decoder_flops(h: int, w: int, c: int = 64, blocks=(3, 3, 3, 1)) -> float:
    """DecoderTiny forward at latent h x w (its input-gradient counts the same)."""
    p = h * w
    f = _conv(p, 4, c)
    for i, nb in enumerate(blocks):
        f += nb * 3 * _conv(p, c, c)
        if i < len(blocks) - 1:
            p *= 4
            f += _conv(p, c, c)
        else:
            f += _conv(p, c, 3)
    return f


def taesd_encoder_flops(h: int, w: int, c: int = 64, blocks=(1, 3, 3, 3)) -> float:
    """EncoderTiny forward producing latent h x w (input 8h x 8w)."""
    p = 64 * h * w
    f = _conv(p, 3, c)
    for i, nb in enumerate(blocks):
        if i > 0:
            p //= 4
            f += _conv(p, c, c)
        f += nb * 3 * _conv(p, c, c)
    return f + _conv(p, c, 4)


def frame_flops(h: int, w: int, steps: int = 50, seeds: int = 1, cfg: UNetConfig = MARIGOLD_V1) -> dict:
    """Algorithmic FLOPs of one frame (all its seeds) at latent h x w with `steps` guided steps."""
    uf, ub = unet_flops(h, w, cfg)
    dec = taesd_decoder_flops(h, w)
    enc = taesd_encoder_flops(h, w)
    step = uf + ub + 2 * dec
    per_seed = steps * step + enc + dec
    return {"unet_fwd": uf, "unet_dgrad": ub, "taesd_dec": dec, "taesd_enc": enc, "per_step": step,
            "per_frame": seeds * per_seed}

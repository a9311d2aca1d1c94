"""Model configuration of the hot path (Marigold v1-0 UNet + TAESD), diffusers-compatible names.

SURVEY.md Appendix A: UNet2DConditionModel, SD2 architecture with 8 input channels
(marigold_dc.py:459 concatenates 4 image + 4 depth latent channels), cross-attention dim 1024
(the [1, 2, 1024] empty-prompt embedding, marigold_dc.py:663-674); AutoencoderTiny (TAESD,
predict.py:484-488).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class UNetConfig:
    in_channels: int = 8
    out_channels: int = 4
    block_out_channels: tuple = (320, 640, 1280, 1280)
    layers_per_block: int = 2
    heads: tuple = (5, 10, 20, 20)
    cross_attention_dim: int = 1024
    norm_num_groups: int = 32
    down_attn: tuple = (True, True, True, False)
    up_attn: tuple = (False, True, True, True)

    @property
    def time_embed_dim(self) -> int:
        return self.block_out_channels[0] * 4


MARIGOLD_V1 = UNetConfig()
TINY = UNetConfig(block_out_channels=(64, 128, 128, 128), heads=(1, 2, 2, 2), cross_attention_dim=64)

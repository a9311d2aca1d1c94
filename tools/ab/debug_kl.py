"""Debug: --vae original pipeline stages vs the oracle (tiny configs, GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_pipeline import synth_inputs  # noqa: E402
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.config import TINY  # noqa: E402
from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline  # noqa: E402
from depth_completion_amd.vae_kl import TINY_KL  # noqa: E402
from oracle import pipeline_ref as P  # noqa: E402
from oracle.diffusers_ref import (DDIMScheduler, UNet2DConditionModel, synthetic_state_dict,  # noqa: E402
                                  synthetic_text_embedding, tiny_unet_config)
from oracle.vae_kl_ref import AutoencoderKL, KLConfig, synthetic_kl_state_dict  # noqa: E402

dev = torch.device("cuda:0")
cfg_o = tiny_unet_config()
imgs, sparses = synth_inputs(1, 48, 64, 60, seed=29)
ocfg = KLConfig(block_out_channels=TINY_KL.block_out_channels, layers_per_block=TINY_KL.layers_per_block)
kl = AutoencoderKL(ocfg)
ksd = synthetic_kl_state_dict(kl, 31)
kl.load_state_dict(ksd)
kl = kl.to(dev)
unet = UNet2DConditionModel(cfg_o)
usd = synthetic_state_dict(unet, 11)
unet.load_state_dict(usd)
emb = synthetic_text_embedding(13, cfg_o.cross_attention_dim)
o = P.OracleMarigoldDC(unet.to(dev), kl, DDIMScheduler(), emb, dtype=torch.float32, device=dev)
pipe = MarigoldDepthCompletionPipeline(usd, ksd, emb, unet_config=TINY, device=dev, vae="original",
                                       vae_config=TINY_KL, use_graph=False)
noise = torch.randn((1, 4, 6, 8), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
# image latents
img = o.image_processor.preprocess(imgs.to(dev), 64, "bilinear", dev, torch.float32)
print(type(img), [getattr(x, "shape", x) for x in (img if isinstance(img, tuple) else (img,))])
for steps in (1, 2, 4):
    for kw in (dict(train_latents=False), dict()):
        d32, l32 = o(imgs.to(dev), sparses.to(dev), 120.0, norm="const", steps=steps, resolution=64, init_noise=noise,
                     **kw)
        dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, norm="const", steps=steps, resolution=64,
                      init_noise=noise, **kw)
        up = pipe._plans[(1, 6, 8)]["unet"]
        il = up.x8[:, :4].float().reshape(1, 6, 8, 4).permute(0, 3, 1, 2)
        print(steps, kw, "dense rel", float((dh - d32).norm() / d32.norm()), "lat rel",
              float((lh.float() - l32.float()).norm() / l32.float().norm()))

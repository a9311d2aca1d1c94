"""Local diffusers-format checkpoints: the construction surface of the reference (predict.py:474-503).

The reference builds its pipeline with ``MarigoldDepthCompletionPipeline.from_pretrained(ckpt,
prediction_type="depth", torch_dtype=dtype)`` and swaps ``pipe.vae = AutoencoderTiny.from_pretrained(...)`` and
``pipe.scheduler = DDIMScheduler.from_config(pipe.scheduler.config, timestep_spacing="trailing")``.  This module
gives the same calls over LOCAL directories (there is no hub access): ``AutoencoderTiny`` / ``AutoencoderKL`` /
``UNet2DConditionModel`` weight holders with ``from_pretrained`` and ``DDIMScheduler.from_config``, read by
``pipeline.MarigoldDepthCompletionPipeline.from_pretrained`` and its ``vae`` / ``scheduler`` setters.

Directory layout (diffusers): ``model_index.json``, ``unet/{config.json, diffusion_pytorch_model.safetensors}``,
``vae/...`` (AutoencoderKL), ``scheduler/scheduler_config.json``, ``text_encoder/{config.json, model.safetensors}``
and ``tokenizer/`` -- the empty-prompt embedding (marigold_dc.py:663-674) is computed once from the CLIP text
encoder (a host-side torch restatement of CLIPTextModel for the 2-token empty prompt, run at load time) and cached
as ``empty_text_embedding.safetensors``, which is also what the native session (dc_load_weights) reads.  A TAESD
checkpoint directory holds ``diffusion_pytorch_model.safetensors`` (+ ``config.json``).
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import torch

from .config import UNetConfig

BOS, EOS = 49406, 49407  # CLIP's <|startoftext|>, <|endoftext|>


def _load_safetensors(path: Path) -> dict:
    from safetensors.torch import load_file
    return load_file(str(path))


def _save_safetensors(sd: dict, path: Path) -> None:
    from safetensors.torch import save_file
    path.parent.mkdir(parents=True, exist_ok=True)
    save_file({k: v.detach().contiguous().cpu() for k, v in sd.items()}, str(path))


def _weights_file(d: Path) -> Path:
    for name in ("diffusion_pytorch_model.safetensors", "diffusion_pytorch_model.fp16.safetensors",
                 "model.safetensors"):
        if (d / name).exists():
            return d / name
    raise FileNotFoundError(f"no safetensors weights in {d}")


def _check_dtype(torch_dtype) -> None:
    if torch_dtype not in (None, torch.bfloat16):
        raise ValueError(f"torch_dtype={torch_dtype}: the HIP sampler runs bf16 (predict.py --precision bf16); "
                         "fp32 is not supported")


# ------------------------------------------------------------------ weight holders (diffusers class names)
class _Weights:
    subfolder = ""

    def __init__(self, state_dict: dict, config: dict | None = None):
        self.state_dict = state_dict
        self.config = dict(config or {})

    @classmethod
    def from_pretrained(cls, path, subfolder: str | None = None, torch_dtype=None, **_):
        _check_dtype(torch_dtype)
        d = Path(path) / (cls.subfolder if subfolder is None else subfolder)
        cfg = json.loads((d / "config.json").read_text()) if (d / "config.json").exists() else {}
        return cls(_load_safetensors(_weights_file(d)), cfg)

    def to(self, *_, **__):
        """``.to("cuda")`` of the reference's call chain: the HIP modules are built on the pipeline's device."""
        return self


class AutoencoderTiny(_Weights):
    """TAESD (``madebyollin/taesd``, predict.py:484-488)."""


class AutoencoderKL(_Weights):
    subfolder = "vae"


class UNet2DConditionModel(_Weights):
    subfolder = "unet"

    def unet_config(self) -> UNetConfig:
        return unet_config_from_dict(self.config)


class DDIMScheduler:
    """Config holder of diffusers.DDIMScheduler; ``from_config(cfg, timestep_spacing="trailing")`` as predict.py:491."""

    def __init__(self, **config):
        self.config = dict(config)

    @classmethod
    def from_config(cls, config: dict, **overrides):
        cfg = dict(config)
        cfg.update(overrides)
        return cls(**cfg)

    @classmethod
    def from_pretrained(cls, path, subfolder: str = "scheduler", **_):
        return cls(**json.loads((Path(path) / subfolder / "scheduler_config.json").read_text()))


class LCMScheduler(DDIMScheduler):
    """``--model lcm`` (predict.py:495-498) is outside the hot path; assigning it to the pipeline raises."""


def kl_config_from_dict(c: dict):
    from .vae_kl import SD_VAE, KLConfig
    if not c:
        return SD_VAE
    return KLConfig(block_out_channels=tuple(c.get("block_out_channels", SD_VAE.block_out_channels)),
                    layers_per_block=c.get("layers_per_block", SD_VAE.layers_per_block),
                    latent_channels=c.get("latent_channels", SD_VAE.latent_channels),
                    scaling_factor=c.get("scaling_factor", SD_VAE.scaling_factor))


def unet_config_from_dict(c: dict) -> UNetConfig:
    if not c:
        return UNetConfig()
    heads = c.get("attention_head_dim", (5, 10, 20, 20))
    ch = tuple(c.get("block_out_channels", (320, 640, 1280, 1280)))
    if isinstance(heads, int):
        heads = (heads,) * len(ch)
    down = tuple("CrossAttn" in t for t in c.get("down_block_types", ["CrossAttnDownBlock2D"] * 3 + ["DownBlock2D"]))
    up = tuple("CrossAttn" in t for t in c.get("up_block_types", ["UpBlock2D"] + ["CrossAttnUpBlock2D"] * 3))
    if c.get("norm_num_groups", 32) != 32:
        raise ValueError("norm_num_groups must be 32")
    return UNetConfig(in_channels=c.get("in_channels", 8), out_channels=c.get("out_channels", 4),
                      block_out_channels=ch, layers_per_block=c.get("layers_per_block", 2), heads=tuple(heads),
                      cross_attention_dim=c.get("cross_attention_dim", 1024), down_attn=down, up_attn=up)


def unet_config_to_dict(cfg: UNetConfig) -> dict:
    n = len(cfg.block_out_channels)
    return {"_class_name": "UNet2DConditionModel", "in_channels": cfg.in_channels, "out_channels": cfg.out_channels,
            "block_out_channels": list(cfg.block_out_channels), "attention_head_dim": list(cfg.heads),
            "cross_attention_dim": cfg.cross_attention_dim, "layers_per_block": cfg.layers_per_block,
            "norm_num_groups": cfg.norm_num_groups,
            "down_block_types": ["CrossAttnDownBlock2D" if a else "DownBlock2D" for a in cfg.down_attn][:n],
            "up_block_types": ["CrossAttnUpBlock2D" if a else "UpBlock2D" for a in cfg.up_attn][:n]}


# ------------------------------------------------------------------ empty-prompt embedding (CLIP text encoder)
def clip_empty_prompt_embedding(sd: dict, config: dict, token_ids=(BOS, EOS)) -> torch.Tensor:
    """CLIPTextModel(input_ids)[0] (last_hidden_state) for the tokenised empty prompt -- marigold_dc.py:664-674,
    tokenizer("", padding="do_not_pad") = [<|startoftext|>, <|endoftext|>].  Host-side fp32 torch restatement of
    transformers' CLIPTextTransformer (pre-LN blocks, causal mask, final LayerNorm), run once at load time; the
    result is a constant of the sampler (it is not on the per-step path).  Returns [1, n_tokens, hidden] fp32."""
    # checkpoints on disk key the weights "text_model.*" (transformers >= 5 drops the prefix in state_dict())
    pre = "text_model." if any(k.startswith("text_model.") for k in sd) else ""
    g = lambda k: sd[pre + k].float()  # noqa: E731
    hidden = config.get("hidden_size", g("embeddings.token_embedding.weight").shape[1])
    heads = config.get("num_attention_heads", 16)
    layers = config.get("num_hidden_layers", sum(1 for k in sd if k.endswith("self_attn.q_proj.weight")))
    eps = config.get("layer_norm_eps", 1e-5)
    act = config.get("hidden_act", "gelu")
    ids = torch.tensor(list(token_ids))
    x = g("embeddings.token_embedding.weight")[ids] + g("embeddings.position_embedding.weight")[: len(ids)]
    x = x[None]
    T = x.shape[1]
    hd = hidden // heads
    mask = torch.full((T, T), float("-inf")).triu(1)

    def ln(t, k):
        return torch.nn.functional.layer_norm(t, (hidden,), g(k + ".weight"), g(k + ".bias"), eps)

    def lin(t, k):
        return t @ g(k + ".weight").t() + g(k + ".bias")

    for i in range(layers):
        p = f"encoder.layers.{i}."
        h = ln(x, p + "layer_norm1")
        q = (lin(h, p + "self_attn.q_proj") * hd ** -0.5).view(1, T, heads, hd).transpose(1, 2)
        k = lin(h, p + "self_attn.k_proj").view(1, T, heads, hd).transpose(1, 2)
        v = lin(h, p + "self_attn.v_proj").view(1, T, heads, hd).transpose(1, 2)
        a = torch.softmax(q @ k.transpose(-1, -2) + mask, dim=-1) @ v
        x = x + lin(a.transpose(1, 2).reshape(1, T, hidden), p + "self_attn.out_proj")
        h = ln(x, p + "layer_norm2")
        h = lin(h, p + "mlp.fc1")
        h = h * torch.sigmoid(1.702 * h) if act == "quick_gelu" else torch.nn.functional.gelu(h)
        x = x + lin(h, p + "mlp.fc2")
    return ln(x, "final_layer_norm")


def empty_text_embedding(path) -> torch.Tensor:
    """The cached empty-prompt embedding of a checkpoint directory, computing (and caching) it from
    text_encoder/ when absent."""
    d = Path(path)
    cache = d / "empty_text_embedding.safetensors"
    if cache.exists():
        return _load_safetensors(cache)["embedding"]
    te = d / "text_encoder"
    cfg = json.loads((te / "config.json").read_text()) if (te / "config.json").exists() else {}
    ids = (BOS, EOS)
    vocab = d / "tokenizer" / "vocab.json"
    if vocab.exists():
        v = json.loads(vocab.read_text())
        ids = (v.get("<|startoftext|>", BOS), v.get("<|endoftext|>", EOS))
    emb = clip_empty_prompt_embedding(_load_safetensors(_weights_file(te)), cfg, ids)
    try:
        _save_safetensors({"embedding": emb}, cache)
    except OSError:
        pass
    return emb


# ------------------------------------------------------------------ writing a checkpoint directory (tests, tools)
def save_pretrained(path, unet_state: dict, unet_cfg: UNetConfig, taesd_state: dict | None = None,
                    text_embedding: torch.Tensor | None = None, vae_state: dict | None = None,
                    text_encoder_state: dict | None = None, text_encoder_config: dict | None = None) -> Path:
    """Write a local diffusers-layout directory (model_index.json, unet/, scheduler/, optional vae/ taesd/
    text_encoder/ and the cached empty_text_embedding.safetensors)."""
    from .pipeline import DDIM_CONFIG
    d = Path(path)
    d.mkdir(parents=True, exist_ok=True)
    (d / "model_index.json").write_text(json.dumps({
        "_class_name": "MarigoldDepthPipeline", "prediction_type": "depth", "unet": ["diffusers", "UNet2DConditionModel"],
        "vae": ["diffusers", "AutoencoderKL"], "scheduler": ["diffusers", "DDIMScheduler"],
        "text_encoder": ["transformers", "CLIPTextModel"], "tokenizer": ["transformers", "CLIPTokenizer"]}, indent=1))
    (d / "unet").mkdir(exist_ok=True)
    (d / "unet" / "config.json").write_text(json.dumps(unet_config_to_dict(unet_cfg), indent=1))
    _save_safetensors(unet_state, d / "unet" / "diffusion_pytorch_model.safetensors")
    (d / "scheduler").mkdir(exist_ok=True)
    sched = dict(DDIM_CONFIG, _class_name="DDIMScheduler", timestep_spacing="leading")  # as shipped; predict.py overrides
    (d / "scheduler" / "scheduler_config.json").write_text(json.dumps(sched, indent=1))
    if taesd_state is not None:
        _save_safetensors(taesd_state, d / "taesd" / "diffusion_pytorch_model.safetensors")
    if vae_state is not None:
        _save_safetensors(vae_state, d / "vae" / "diffusion_pytorch_model.safetensors")
    if text_encoder_state is not None:
        (d / "text_encoder").mkdir(exist_ok=True)
        (d / "text_encoder" / "config.json").write_text(json.dumps(text_encoder_config or {}, indent=1))
        _save_safetensors(text_encoder_state, d / "text_encoder" / "model.safetensors")
    if text_embedding is not None:
        _save_safetensors({"embedding": text_embedding.reshape(1, -1, text_embedding.shape[-1]).float()},
                          d / "empty_text_embedding.safetensors")
    return d


def synthetic_clip_state(hidden: int, layers: int, inter: int, seed: int = 21, vocab: int = 49408,
                         positions: int = 77) -> dict:
    """Seeded CLIP text-encoder weights in transformers' key layout (tests; there are no checkpoints offline)."""
    g = torch.Generator().manual_seed(seed)

    def w(*shape):
        return (torch.rand(*shape, generator=g) * 2 - 1) / math.sqrt(shape[-1])

    sd = {"text_model.embeddings.token_embedding.weight": torch.randn(vocab, hidden, generator=g) * 0.02,
          "text_model.embeddings.position_embedding.weight": torch.randn(positions, hidden, generator=g) * 0.01}
    for i in range(layers):
        p = f"text_model.encoder.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            sd[p + f"self_attn.{n}.weight"] = w(hidden, hidden)
            sd[p + f"self_attn.{n}.bias"] = w(hidden) * 0.1
        for n in ("layer_norm1", "layer_norm2"):
            sd[p + n + ".weight"] = 1 + 0.1 * w(hidden)
            sd[p + n + ".bias"] = 0.1 * w(hidden)
        sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"] = w(inter, hidden), 0.1 * w(inter)
        sd[p + "mlp.fc2.weight"], sd[p + "mlp.fc2.bias"] = w(hidden, inter), 0.1 * w(hidden)
    sd["text_model.final_layer_norm.weight"] = 1 + 0.1 * w(hidden)
    sd["text_model.final_layer_norm.bias"] = 0.1 * w(hidden)
    return sd

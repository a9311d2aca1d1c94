"""The native session (include/dcamd.h "native session", csrc/session.cpp) against the Python pipeline (GPU).

Both hosts pack the same weights, allocate the same buffers and launch the same kernels with the same arguments
and GEMM variants, so every output must be BITWISE equal:
* dc_complete (encode + guided loop + final decode in one call) vs MarigoldDepthCompletionPipeline.__call__;
* dc_encode -> dc_guided_sample -> dc_decode_dense vs dc_complete;
* graph replay vs eager (use_graph 0), and a second frame on the captured graph (tables refreshed in place);
* the reference construction chain (predict.py:474-494): from_pretrained(dir) with the AutoencoderKL of vae/,
  then ``pipe.vae = AutoencoderTiny.from_pretrained(...)`` and the trailing-spacing scheduler swap;
* the ValueError of an empty sparse mask (marigold_dc.py:97-98) as a status + message.
Tiny UNet at 96x128 / res 128 (sparse-aware decode active), and the full Marigold v1-0 UNet at the C2 shape
(768x576, 500 points) for 3 guided steps.
"""
import pytest
import torch

from depth_completion_amd import pretrained as pt
from depth_completion_amd import synthetic
from depth_completion_amd.config import MARIGOLD_V1, TINY
from depth_completion_amd.native import NativeSession, SampleParams
from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
from test_gpu_pipeline import synth_inputs

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")


def _noise(seed, h, w):
    return torch.randn((1, 4, h, w), generator=torch.Generator().manual_seed(seed), dtype=torch.bfloat16)


@pytest.fixture(scope="module")
def tiny_dir(tmp_path_factory):
    from depth_completion_amd.vae_kl import TINY_KL
    d = tmp_path_factory.mktemp("tiny_ckpt")
    pt.save_pretrained(d, synthetic.unet_state_dict(TINY, 11), TINY, taesd_state=synthetic.taesd_state_dict(12),
                       text_embedding=synthetic.text_embedding(13, TINY.cross_attention_dim),
                       vae_state=synthetic.kl_state_dict(TINY_KL, 12))
    import json
    (d / "vae" / "config.json").write_text(json.dumps({"block_out_channels": list(TINY_KL.block_out_channels),
                                                       "layers_per_block": TINY_KL.layers_per_block}))
    return d


def _reference_chain(d):
    """predict.py:474-494 over the local directory."""
    pipe = MarigoldDepthCompletionPipeline.from_pretrained(d, prediction_type="depth",
                                                           torch_dtype=torch.bfloat16).to("cuda")
    assert pipe.vae_kind == "original"
    pipe.vae = pt.AutoencoderTiny.from_pretrained(d / "taesd", torch_dtype=torch.bfloat16).to("cuda")
    pipe.scheduler = pt.DDIMScheduler.from_config(pipe.scheduler.config, timestep_spacing="trailing")
    return pipe


def test_session_equals_python_pipeline_tiny(tiny_dir):
    imgs, sparses = synth_inputs(2, 96, 128, 60, seed=3)
    h, w = MarigoldDepthCompletionPipeline.latent_hw(96, 128, 128)
    noise = _noise(2024, h, w)
    kw = dict(norm="const", steps=3, resolution=128)
    pipe = _reference_chain(tiny_dir)
    direct = MarigoldDepthCompletionPipeline(synthetic.unet_state_dict(TINY, 11), synthetic.taesd_state_dict(12),
                                             synthetic.text_embedding(13, TINY.cross_attention_dim), unet_config=TINY,
                                             device=dev)
    dp, lp = pipe(imgs.to(dev), sparses.to(dev), 120.0, init_noise=noise, **kw)
    dd, ld = direct(imgs.to(dev), sparses.to(dev), 120.0, init_noise=noise, **kw)
    assert torch.equal(dp, dd) and torch.equal(lp, ld)        # from_pretrained chain == direct construction
    s = NativeSession(tiny_dir, dev)
    prm = SampleParams.make(norm="const", steps=3, resolution=128)
    dn, ln = s.complete(imgs, sparses, noise, prm)
    torch.cuda.synchronize()
    assert torch.equal(ln, lp), (ln.float() - lp.float()).abs().max()
    assert torch.equal(dn, dp), (dn - dp).abs().max()
    # the three-call form
    lat_img = s.encode(imgs, resolution=128)
    lat, aff = s.guided_sample(lat_img, sparses, noise, prm)
    dense = s.decode_dense(lat, aff, sparses, prm)
    assert torch.equal(lat, ln) and torch.equal(dense, dn)
    # eager (no graph) == graph
    de, le = s.complete(imgs, sparses, noise, SampleParams.make(norm="const", steps=3, resolution=128,
                                                                use_graph=False))
    assert torch.equal(le, ln) and torch.equal(de, dn)
    # another frame pair on the captured graph; minmax norm, SGD; and a warm start from the previous latents
    imgs2, sparses2 = synth_inputs(2, 96, 128, 55, seed=4)
    k2 = dict(norm="minmax", steps=3, resolution=128, opt="sgd")
    dp2, lp2 = pipe(imgs2.to(dev), sparses2.to(dev), 120.0, init_noise=noise, pred_latents_prev=lp, **k2)
    dn2, ln2 = s.complete(imgs2, sparses2, noise, SampleParams.make(**k2), prev=ln)
    torch.cuda.synchronize()
    assert torch.equal(ln2, lp2) and torch.equal(dn2, dp2)


def test_session_errors(tiny_dir):
    s = NativeSession(tiny_dir, dev)
    imgs, sparses = synth_inputs(1, 96, 128, 40, seed=5)
    h, w = s.latent_hw(96, 128, 128)
    with pytest.raises(ValueError, match="No valid values found in mask"):
        s.complete(imgs, torch.zeros_like(sparses), _noise(1, h, w), SampleParams.make(steps=2, resolution=128))
    bad = SampleParams.make(steps=2, resolution=128)
    bad.beta = 1.5
    with pytest.raises(ValueError, match="beta"):
        s.complete(imgs, sparses, _noise(1, h, w), bad)
    bad = SampleParams.make(steps=2, resolution=128, projection="log", min_depth=0.0)
    with pytest.raises(ValueError, match="min_depth"):
        s.complete(imgs, sparses, _noise(1, h, w), bad)
    # still usable after the errors
    d, _ = s.complete(imgs, sparses, _noise(1, h, w), SampleParams.make(steps=2, resolution=128))
    assert torch.isfinite(d).all()


def test_session_memory_flat_and_failed_reload(tiny_dir, tmp_path):
    """A long-running session over mixed input sizes, step counts and weight reloads keeps its device memory
    flat (every DevMem reassignment frees the blocks it replaces), and a reload that fails partway leaves the
    session unloaded -- the next call reports "no weights loaded" instead of launching on stale pointers."""
    s = NativeSession(tiny_dir, dev)
    shapes = ((96, 128), (192, 256))   # same 12 x 16 latent plan at resolution 128, different H * W tables
    noise = _noise(2024, 12, 16)
    inputs = {hw: synth_inputs(1, hw[0], hw[1], 40, seed=6) for hw in shapes}

    def sweep():
        for hw in shapes:
            for steps in (2, 3):
                imgs, sparses = inputs[hw]
                d, _ = s.complete(imgs, sparses, noise, SampleParams.make(steps=steps, resolution=128))
                lat = torch.zeros(1, 4, 12, 16, dtype=torch.bfloat16, device=dev)
                aff = torch.tensor([[1.0, 0.0]], device=dev)
                s.decode_dense(lat, aff, sparses, SampleParams.make(steps=steps, resolution=128))
        s._check(s.lib.dc_load_weights(s.h, str(tiny_dir).encode(), b""), "dc_load_weights")
        torch.cuda.synchronize()

    sweep()
    free0 = torch.cuda.mem_get_info(dev)[0]
    for _ in range(3):
        sweep()
    free1 = torch.cuda.mem_get_info(dev)[0]
    print(f"\nsession device memory over 3 sweeps: {(free0 - free1) / 2**20:+.1f} MiB")
    assert free0 - free1 < 8 << 20, (free0, free1)
    # a reload refused by its config checks (no unet/config.json: the Marigold defaults do not match the tiny
    # embedding) changes nothing: the session keeps its weights
    bad = tmp_path / "bad"
    (bad / "unet").mkdir(parents=True)
    import shutil
    shutil.copy(tiny_dir / "empty_text_embedding.safetensors", bad / "empty_text_embedding.safetensors")
    with pytest.raises(Exception):
        s._check(s.lib.dc_load_weights(s.h, str(bad).encode(), b""), "dc_load_weights")
    imgs, sparses = inputs[shapes[0]]
    d, _ = s.complete(imgs, sparses, noise, SampleParams.make(steps=2, resolution=128))
    assert torch.isfinite(d).all()
    # a reload that fails partway (config fine, no UNet safetensors) leaves the session unloaded
    shutil.copy(tiny_dir / "unet" / "config.json", bad / "unet" / "config.json")
    with pytest.raises(Exception):
        s._check(s.lib.dc_load_weights(s.h, str(bad).encode(), b""), "dc_load_weights")
    with pytest.raises(ValueError, match="no weights loaded"):
        s.complete(imgs, sparses, noise, SampleParams.make(steps=2, resolution=128))
    # ... and a good reload makes it usable again
    s._check(s.lib.dc_load_weights(s.h, str(tiny_dir).encode(), b""), "dc_load_weights")
    d, _ = s.complete(imgs, sparses, noise, SampleParams.make(steps=2, resolution=128))
    assert torch.isfinite(d).all()
    with pytest.raises(ValueError):
        s.decode_dense(torch.zeros(1, 4, 12, 16, dtype=torch.bfloat16, device=dev), torch.zeros(1, 2, device=dev),
                       torch.zeros(1, 1, 0, 0, device=dev), SampleParams.make(steps=2, resolution=128))


def test_session_equals_python_pipeline_c2_full_unet(tmp_path):
    """Full Marigold v1-0 UNet at the C2 shape (latent 72x96, tuned GEMM table, stream-K attention, sparse-aware
    decode), 3 guided steps: bitwise equal."""
    d = tmp_path / "full"
    usd = {k: v.to(torch.bfloat16) for k, v in synthetic.unet_state_dict(MARIGOLD_V1, 11).items()}
    pt.save_pretrained(d, usd, MARIGOLD_V1, taesd_state=synthetic.taesd_state_dict(12),
                       text_embedding=synthetic.text_embedding(13, 1024))
    imgs, sparses = synth_inputs(1, 576, 768, 500, seed=41)
    noise = _noise(2024, 72, 96)
    pipe = MarigoldDepthCompletionPipeline.from_pretrained(d)
    pipe.scheduler = pt.DDIMScheduler.from_config(pipe.scheduler.config, timestep_spacing="trailing")
    dp, lp = pipe(imgs.to(dev), sparses.to(dev), 120.0, norm="const", steps=3, resolution=768, init_noise=noise)
    del pipe
    torch.cuda.empty_cache()
    s = NativeSession(d, dev)
    dn, ln = s.complete(imgs, sparses, noise, SampleParams.make(norm="const", steps=3, resolution=768))
    torch.cuda.synchronize()
    assert torch.equal(ln, lp), (ln.float() - lp.float()).abs().max()
    assert torch.equal(dn, dp), (dn - dp).abs().max()

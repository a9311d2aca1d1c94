"""Parity of the HIP guided sampler at the BASELINE.json workloads themselves (GPU).

* C2: one 768x576 frame, 500 points, the full Marigold v1-0 UNet, 50 guided steps, norm="const" -- the
  headline config (latent 72x96: T = 6912 tokens at level 0, the tuned GEMM table, stream-K attention
  backward, the sparse-aware decode), against the fp32 oracle (oracle/pipeline_ref.py on PyTorch-ROCm)
  after the reference's closed-form fit (compute_affine_params, marigold_dc.py:53-128).  Bound: at most
  2x the oracle's own bf16 execution's error (+1e-3) -- 50 chained bf16 Adam + DDIM steps amplify
  rounding identically in both -- and below the absolute 5 % mean / 19 % p99 of the frame's depth range.
* C3: the same frame inside a batch of 8 (batched MFMA path, M = 8 x 6912): frame 0 of the batch-8 call against
  the fp32 oracle's 50-step run of that frame (the C2 bounds), and -- frames never interact (marigold_dc.py:877) --
  frames 0 / 3 / 7 against their own single-frame runs within the same bf16 bound.
* C1: a 384x384 image at processing resolution 768 (latent 96x96, T = 9216 -- a shape the tuned table
  never saw), 100 points, 10 guided steps.
* C5: the 10-seed ensemble (seeds 2024..2033) + affine fit at the 1600x900 shape, tiny UNet, against the
  oracle's per-seed loop + mean + compute_affine_params; and dc_ensemble_fit alone against the
  reference's compute_affine_params on identical inputs.
Every test prints the measured errors.
"""
import pytest
import torch

from oracle import pipeline_ref as P
from oracle.diffusers_ref import UNetConfig, tiny_unet_config
from test_gpu_pipeline import build, fitted_error, synth_inputs

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")


def _noise(seed, eh, ew):
    return torch.randn((1, 4, eh, ew), generator=torch.Generator().manual_seed(seed), dtype=torch.bfloat16)


def _lat_err(a, ref):
    return float((a.float().cpu() - ref.float().cpu()).norm() / ref.float().cpu().norm())


@pytest.fixture(scope="module")
def full_c2():
    """fp32 / bf16 oracle and the HIP pipeline on the full UNet, C2 frame 0 (shared by the C2 / C3 tests)."""
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    imgs, sparses = synth_inputs(8, 576, 768, 500, seed=41)
    kw = dict(norm="const", steps=50, resolution=768, init_noise=_noise(2024, 72, 96))
    o32, usd, vsd, emb = build(UNetConfig(), MARIGOLD_V1, torch.float32, dev)
    trace = []   # the fp32 trajectory, step by step (teacher-forced test)
    d32, l32 = o32(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, step_hook=_recorder(trace), **kw)
    del o32
    o16, *_ = build(UNetConfig(), MARIGOLD_V1, torch.bfloat16, dev)
    d16, l16 = o16(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
    del o16
    torch.cuda.empty_cache()
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    return dict(imgs=imgs, sparses=sparses, kw=kw, d32=d32.cpu(), l32=l32.cpu(), d16=d16.cpu(), l16=l16.cpu(),
                pipe=pipe, usd=usd, vsd=vsd, emb=emb, trace=trace)


def _adam_state(optim, p):
    st = optim.state.get(p, {})
    return {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}


def _recorder(trace):
    """oracle step_hook recording the state entering every guided step (latent, image latents, Adam state of the
    latent and of the learned affine) and what the step produced (v, the rescaled gradient, the new latent)."""
    def hook(phase, i, t, st):
        lat, optim = st["lat"], st["optim"]
        if phase == "pre":
            s, sh = st["aff"]
            trace.append(dict(i=i, t=int(t), lat=lat.detach().clone(), img_lat=st["img_lat"].detach().clone(),
                              adam=_adam_state(optim, lat), aff=(s.detach().clone(), sh.detach().clone()),
                              adam_aff=(_adam_state(optim, s), _adam_state(optim, sh))))
        else:
            trace[-1].update(v=st["v"].clone(), grad=st["grad"].clone(), post=lat.detach().clone())
    return hook


def _forcer(trace, out, dtype):
    """oracle step_hook that replays ``trace`` one step at a time: each step starts from the recorded state
    (cast to this execution's dtype) and what it produces is stored in ``out``."""
    def hook(phase, i, t, st):
        lat, optim = st["lat"], st["optim"]
        r = trace[i]
        if phase == "pre":
            lat.data.copy_(r["lat"].to(lat.dtype))
            st["img_lat"] = r["img_lat"].to(dtype)
            for p, src, sv in ((lat, r["adam"], None), (st["aff"][0], r["adam_aff"][0], r["aff"][0]),
                               (st["aff"][1], r["adam_aff"][1], r["aff"][1])):
                if sv is not None:
                    p.data.copy_(sv)
                optim.state.pop(p, None)
                if src:
                    optim.state[p] = {k: (v.clone().to(p.dtype) if torch.is_tensor(v) and v.dim() else
                                          (v.clone() if torch.is_tensor(v) else v)) for k, v in src.items()}
        else:
            out.append(dict(v=st["v"].clone(), grad=st["grad"].clone(), post=lat.detach().clone()))
    return hook


def _rel(a, ref):
    a, ref = a.float().cpu().flatten(), ref.float().cpu().flatten()
    return float((a - ref).norm() / ref.norm().clamp(min=1e-30))


def test_c2_teacher_forced_per_step(full_c2):
    """Per-step parity at C2 without the chaotic 50-step amplification: at each of the 50 trailing timesteps the
    HIP step and the bf16 oracle step both start from the fp32 oracle's state entering that step (latent, image
    latents, Adam state of the latent and of the learned affine, step counter) and are compared with the fp32
    oracle's step on v (UNet output), the latent gradient after the ||eps|| / ||g|| rescale, and the latent after
    Adam + the DDIM update (marigold_dc.py:807-904).

    Measured on MI355X (profiles/r03b/c2_teacher_forced.txt), relative L2 over the frame: v 1.37-1.62 % (bf16
    oracle 1.51-1.87 %), new latent 0.39-2.91 % (bf16 oracle 0.40-2.91 %; 2.9 % at t = 999, where Adam's first
    step moves every element by +-lr on the sign of the gradient), gradient 25-55 % (bf16 oracle 26-76 %: the
    point-loss gradient through a bf16 UNet backward is itself that noisy).  Bounds, every step: v <= 2 % and
    <= 1.25x the bf16 oracle's + 1e-3; new latent <= 3.5 % and <= 1.25x the bf16 oracle's + 1e-3; gradient
    <= 2x the bf16 oracle's + 2e-2."""
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    f = full_c2
    trace = f["trace"]
    assert len(trace) == 50 and all("post" in r for r in trace)
    img, sp = f["imgs"][:1].to(dev), f["sparses"][:1].to(dev)
    # bf16 oracle forced along the fp32 trajectory
    o16, *_ = build(UNetConfig(), MARIGOLD_V1, torch.bfloat16, dev)
    b16 = []
    o16(img, sp, 120.0, step_hook=_forcer(trace, b16, torch.bfloat16), **f["kw"])
    del o16
    torch.cuda.empty_cache()
    # HIP: an eager pipeline set up by a full call (tables, plans, decode row lists), then one step per timestep
    pipe = MarigoldDepthCompletionPipeline(f["usd"], f["vsd"], f["emb"], unet_config=MARIGOLD_V1, device=dev,
                                           use_graph=False)
    pipe(img, sp, 120.0, **f["kw"])
    st = pipe._plans[(1, 72, 96)]
    st["dec"].set_rows(st.get("row_sets"))   # the guided steps' sparse-aware decode
    up = st["unet"]
    P = 72 * 96

    def nhwc(x):   # [1, 4, h, w] -> [P, 4]
        return x.detach().to(dev, torch.bfloat16).permute(0, 2, 3, 1).reshape(P, 4)

    def nchw(x):   # [P, 4] -> [1, 4, h, w]
        return x.reshape(1, 72, 96, 4).permute(0, 3, 1, 2).float().cpu()

    rows = []
    for r, b in zip(trace, b16):
        i = r["i"]
        up.x8[:, 0:4] = nhwc(r["img_lat"])
        up.x8[:, 4:8] = nhwc(r["lat"])
        ad = r["adam"]
        st["m_lat"].view(P, 4).copy_(nhwc(ad["exp_avg"]) if ad else 0)
        st["v_lat"].view(P, 4).copy_(nhwc(ad["exp_avg_sq"]) if ad else 0)
        st["affine"].copy_(torch.tensor([[float(r["aff"][0]), float(r["aff"][1])]]))
        for j, a in enumerate(r["adam_aff"]):
            st["m_aff"][0, j] = float(a["exp_avg"]) if a else 0.0
            st["v_aff"][0, j] = float(a["exp_avg_sq"]) if a else 0.0
        pipe.ctx.step.fill_(i)
        pipe._step(st)
        torch.cuda.synchronize()
        v_h = nchw(up.v[:, 0:4])
        g_raw = (st["gdir"][:, 0:4].float() + up.gx[:, 0:4].float()).to(torch.bfloat16).float()
        factor = float(st["dbg"][0, 1])
        g_h = nchw(g_raw * factor)
        x_h = nchw(up.x8[:, 4:8])
        e = (_rel(v_h, r["v"]), _rel(g_h, r["grad"]), _rel(x_h, r["post"]))
        eb = (_rel(b["v"], r["v"]), _rel(b["grad"], r["grad"]), _rel(b["post"], r["post"]))
        rows.append((i, r["t"], e, eb))
    print("\nC2 teacher-forced per-step relative errors vs the fp32 oracle (HIP | oracle-bf16):")
    print("step    t     v(HIP)  v(bf16)   grad(HIP) grad(bf16)  lat(HIP)  lat(bf16)")
    for i, t, e, eb in rows:
        print(f"{i:4d} {t:5d}   {e[0]:.5f}  {eb[0]:.5f}   {e[1]:.5f}   {eb[1]:.5f}    {e[2]:.5f}   {eb[2]:.5f}")
    worst = [max(r[2][k] for r in rows) for k in range(3)]
    worst_b = [max(r[3][k] for r in rows) for k in range(3)]
    print(f"worst over 50 steps: v {worst[0]:.5f} ({worst_b[0]:.5f}) grad {worst[1]:.5f} ({worst_b[1]:.5f}) "
          f"latent {worst[2]:.5f} ({worst_b[2]:.5f})")
    for i, t, e, eb in rows:
        assert e[0] <= 0.02 and e[0] <= 1.25 * eb[0] + 1e-3, (i, t, e, eb)
        assert e[1] <= 2 * eb[1] + 2e-2, (i, t, e, eb)
        assert e[2] <= 0.035 and e[2] <= 1.25 * eb[2] + 1e-3, (i, t, e, eb)


def test_c2_full_unet_50_steps(full_c2):
    f = full_c2
    dh, lh = f["pipe"](f["imgs"][:1].to(dev), f["sparses"][:1].to(dev), 120.0, **f["kw"])
    torch.cuda.synchronize()
    assert dh.shape == (1, 1, 576, 768) and lh.shape == (1, 4, 72, 96) and torch.isfinite(dh).all()
    sp = f["sparses"][:1]
    mean_h, p99_h = fitted_error(dh, f["d32"], sp)
    mean_b, p99_b = fitted_error(f["d16"], f["d32"], sp)
    lat_h, lat_b = _lat_err(lh, f["l32"]), _lat_err(f["l16"], f["l32"])
    print(f"\nC2 (full UNet, 768x576, 500 pts, 50 steps): HIP fitted |d| mean {mean_h:.5f} p99 {p99_h:.5f} "
          f"latent {lat_h:.4f} | oracle-bf16 mean {mean_b:.5f} p99 {p99_b:.5f} latent {lat_b:.4f}")
    # 50 chained bf16 Adam + DDIM steps on synthetic weights: the reference's own bf16 execution drifts from
    # its fp32 one by 3.86 % mean / 14.5 % p99 of the range here (chaotic guidance: Adam's first steps move
    # every latent by +-lr on the sign of a gradient near zero); per step the HIP path is as close to the fp32
    # oracle as the bf16 oracle is (test_c2_teacher_forced_per_step).  Bounds: relative to that drift, and the
    # stated absolute C2 tolerance -- fitted per-pixel |depth diff| <= 5 % mean / 19 % p99 of the frame's depth
    # range (measured HIP 3.91 % / 14.8 %, profiles/r03b/; ~28 % headroom).  Why 10x SURVEY's proposed 0.5 % / 2 %:
    # that figure is below the reference path's own bf16-vs-fp32 drift at this workload (the bf16 oracle is 3.86 % /
    # 14.5 % from the fp32 oracle after 50 guided steps), so no bf16 implementation -- the reference's included --
    # can meet it end to end; the absolute bound sits ~1.3x above that drift, and the per-step bound (each step from
    # the fp32 oracle's state, within 1.25x the bf16 oracle's own per-step error) is test_c2_teacher_forced_per_step
    assert mean_h <= 2 * mean_b + 1e-3 and p99_h <= 2 * p99_b + 1e-3
    assert mean_h <= 0.05 and p99_h <= 0.19
    assert lat_h <= 2 * lat_b + 2e-3


def test_c2_graph_replay_new_frames_equal_eager(full_c2):
    """At the C2 shape: calls on new frames replay the step graph captured by the first call (tables and
    decode row lists refreshed in place), and a call with another step count recaptures it; every call equals
    an eager (un-captured) pipeline's bitwise.  (A hipMemsetAsync captured in the step graph did not clear the
    1.7 MB dA map on replay in a later call; 3-step calls keep this short.)"""
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    f = full_c2
    pipe = f["pipe"]
    eager = MarigoldDepthCompletionPipeline(f["usd"], f["vsd"], f["emb"], unet_config=MARIGOLD_V1, device=dev,
                                            use_graph=False)
    imgs, sparses = f["imgs"], f["sparses"]
    kw = dict(f["kw"], steps=3)
    for i, steps in ((1, 3), (2, 3), (1, 4), (3, 4), (2, 3)):
        k = dict(kw, steps=steps)
        dg, lg = pipe(imgs[i:i + 1].to(dev), sparses[i:i + 1].to(dev), 120.0, **k)
        de, le = eager(imgs[i:i + 1].to(dev), sparses[i:i + 1].to(dev), 120.0, **k)
        torch.cuda.synchronize()
        assert torch.equal(lg, le) and torch.equal(dg, de), (i, steps)


def test_c3_batch8_frames_equal_single_runs(full_c2):
    """Batch 8 through the batched path: each frame vs its own batch-1 run (same initial noise, which the
    reference shares across the batch, marigold_dc.py:677-684); bound = the bf16 oracle's C2 error."""
    f = full_c2
    pipe = f["pipe"]
    imgs, sparses = f["imgs"], f["sparses"]
    db, lb = pipe(imgs.to(dev), sparses.to(dev), 120.0, **f["kw"])
    torch.cuda.synchronize()
    assert db.shape == (8, 1, 576, 768) and lb.shape == (8, 4, 72, 96) and torch.isfinite(db).all()
    db, lb = db.cpu(), lb.cpu()
    mean_b, p99_b = fitted_error(f["d16"], f["d32"], sparses[:1])
    lat_b = _lat_err(f["l16"], f["l32"])
    # the batch-8 call's frame 0 against the fp32 oracle's own 50-step run of that frame (the C2 bounds)
    m0, p0 = fitted_error(db[0:1], f["d32"], sparses[:1])
    l0 = _lat_err(lb[0:1], f["l32"])
    print(f"\nC3 frame 0 vs the fp32 oracle: fitted |d| mean {m0:.5f} p99 {p0:.5f} latent {l0:.4f} | oracle-bf16 "
          f"mean {mean_b:.5f} p99 {p99_b:.5f} latent {lat_b:.4f}")
    assert m0 <= 2 * mean_b + 1e-3 and p0 <= 2 * p99_b + 1e-3 and l0 <= 2 * lat_b + 2e-3
    assert m0 <= 0.05 and p0 <= 0.19
    worst = (0.0, 0.0, 0.0)
    for i in (0, 3, 7):
        ds, ls = pipe(imgs[i:i + 1].to(dev), sparses[i:i + 1].to(dev), 120.0, **f["kw"])
        m, p99 = fitted_error(db[i:i + 1], ds.cpu(), sparses[i:i + 1])
        la = _lat_err(lb[i:i + 1], ls)
        print(f"\nC3 frame {i}: batch-8 vs single fitted |d| mean {m:.5f} p99 {p99:.5f} latent {la:.4f}")
        worst = tuple(max(a, b) for a, b in zip(worst, (m, p99, la)))
        assert m <= 2 * mean_b + 1e-3 and p99 <= 2 * p99_b + 1e-3 and la <= 2 * lat_b + 2e-3
    print(f"C3 worst over frames 0/3/7: mean {worst[0]:.5f} p99 {worst[1]:.5f} latent {worst[2]:.4f} "
          f"(bound from the bf16 oracle: mean {2 * mean_b + 1e-3:.5f} p99 {2 * p99_b + 1e-3:.5f})")


def test_c1_384_at_768_10_steps():
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    imgs, sparses = synth_inputs(1, 384, 384, 100, seed=0)
    kw = dict(norm="const", steps=10, resolution=768, init_noise=_noise(2024, 96, 96))
    o32, usd, vsd, emb = build(UNetConfig(), MARIGOLD_V1, torch.float32, dev)
    d32, l32 = o32(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    del o32
    o16, *_ = build(UNetConfig(), MARIGOLD_V1, torch.bfloat16, dev)
    d16, l16 = o16(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    del o16
    torch.cuda.empty_cache()
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    torch.cuda.synchronize()
    assert dh.shape == (1, 1, 384, 384) and lh.shape == (1, 4, 96, 96) and torch.isfinite(dh).all()
    mean_h, p99_h = fitted_error(dh, d32, sparses)
    mean_b, p99_b = fitted_error(d16, d32, sparses)
    lat_h, lat_b = _lat_err(lh, l32), _lat_err(l16, l32)
    print(f"\nC1 (384x384 @ 768, latent 96x96, 10 steps): HIP fitted |d| mean {mean_h:.5f} p99 {p99_h:.5f} "
          f"latent {lat_h:.4f} | oracle-bf16 mean {mean_b:.5f} p99 {p99_b:.5f} latent {lat_b:.4f}")
    assert mean_h <= 2 * mean_b + 1e-3 and p99_h <= 2 * p99_b + 1e-3
    assert mean_h <= 0.02 and p99_h <= 0.08
    assert lat_h <= 2 * lat_b + 2e-3


def test_ensemble_fit_kernel_matches_reference_fit():
    """dc_ensemble_fit on identical inputs: mean over seeds, then compute_affine_params (fp64 sums on the
    device; the reference's fp32 torch sums differ by rounding only)."""
    from depth_completion_amd import _lib
    g = torch.Generator().manual_seed(3)
    n, S, H, W = 3, 10, 90, 160
    dense = torch.rand(n * S, 1, H, W, generator=g) * 50 + 5
    sp = torch.where(torch.rand(n, 1, H, W, generator=g) < 0.02, torch.rand(n, 1, H, W, generator=g) * 80 + 2,
                     torch.zeros(()))
    mean = dense.view(n, S, 1, H, W).double().mean(1)
    sc, sh = P.compute_affine_params(mean, sp.double(), sp > 0)
    ref = mean * sc.view(-1, 1, 1, 1) + sh.view(-1, 1, 1, 1)
    lib = _lib.load()
    nws = lib.dc_ensemble_ws_bytes(n, H * W)
    ws = torch.empty(-(-nws // 8), dtype=torch.float64, device=dev)
    out = torch.empty(n, 1, H, W, device=dev)
    aff = torch.empty(n, 2, device=dev)
    dd, spd = dense.to(dev), sp.to(dev)
    _lib.call("dc_ensemble_fit", dd.data_ptr(), n, S, H * W, spd.data_ptr(), out.data_ptr(), aff.data_ptr(),
              ws.data_ptr(), nws, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    torch.testing.assert_close(aff[:, 0].double().cpu(), sc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(aff[:, 1].double().cpu(), sh, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-5, atol=1e-4)


def test_c5_ensemble_10_seeds():
    """C5 shape (1600x900 at resolution 768: latent 54x96, 3000 points) with the 10-seed ensemble, tiny UNet,
    3 guided steps: HIP ensemble() (one batched call of 10 seeds) vs the oracle's per-seed loop."""
    from depth_completion_amd.config import TINY
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    h, w = 900, 1600
    imgs, sparses = synth_inputs(1, h, w, 3000, seed=50)
    seeds = list(range(2024, 2034))
    noises = [_noise(s, 54, 96) for s in seeds]
    kw = dict(norm="const", steps=3, resolution=768)
    cfg_o = tiny_unet_config()
    o32, usd, vsd, emb = build(cfg_o, TINY, torch.float32, dev)
    r32, *_ = P.ensemble(o32, imgs.to(dev), sparses.to(dev), 120.0, noises, **kw)
    o16, *_ = build(cfg_o, TINY, torch.bfloat16, dev)
    r16, *_ = P.ensemble(o16, imgs.to(dev), sparses.to(dev), 120.0, noises, **kw)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=TINY, device=dev)
    dh, aff, lat = pipe.ensemble(imgs.to(dev), sparses.to(dev), 120.0, seeds=seeds, **kw)
    torch.cuda.synchronize()
    assert dh.shape == (1, 1, h, w) and aff.shape == (1, 2) and lat.shape == (10, 4, 54, 96)
    assert torch.isfinite(dh).all()
    rng = float(r32.max() - r32.min())
    err_h = float((dh.cpu() - r32.cpu()).abs().mean()) / rng
    err_b = float((r16.cpu() - r32.cpu()).abs().mean()) / rng
    print(f"\nC5 10-seed ensemble (tiny UNet, 3 steps): HIP |d| {err_h:.5f} of range | oracle-bf16 {err_b:.5f}")
    assert err_h <= 2 * err_b + 2e-3
    # the seeds really differ (else the ensemble would be one sample ten times)
    assert float((lat[0].float() - lat[1].float()).abs().mean()) > 1e-2


def _kitti_frames(n, seed):
    """C4 frames: 1216x352 RGB + a 64-beam-like LiDAR pattern (64 scan rows evenly spaced over the lower 60 % of
    the image, each pixel kept with p = 0.25, 8-bit quantised depth), a different pattern per frame."""
    h, w = 352, 1216
    imgs, _ = synth_inputs(n, h, w, 0, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, h), torch.linspace(0, 1, w), indexing="ij")
    sps = []
    for i in range(n):
        rows = torch.linspace(0.4 * h, h - 1, 64).round().long()
        keep = torch.zeros(h, w, dtype=torch.bool)
        keep[rows] = torch.rand(64, w, generator=g) < 0.25
        field = ((10 + 80 * yy + 20 * torch.sin(6.28 * xx + i)) * 255 / 120).round().clamp(1, 255) * 120 / 255
        sps.append(torch.where(keep, field, torch.zeros(()))[None])
    return imgs, torch.stack(sps)


@pytest.mark.parametrize("nb", [1, 8])
def test_c4_full_unet_3_steps(nb):
    """C4 (KITTI 1216x352 at resolution 768: resized 222x768, padded to latent 28x96, 64-beam LiDAR) through the
    FULL Marigold v1-0 UNet, 3 guided steps, one frame and a batch of 8 frames (the batched MFMA path at M =
    8 x 2688 rows, the nearest-tuned-shape GEMM variants), against the fp32 oracle after the closed-form fit.
    Bound: 2x the bf16 oracle's own error + 2e-3 (fitted |d|, per frame) and 2 % mean / 8 % p99 absolute."""
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    imgs, sparses = _kitti_frames(nb, seed=60)
    kw = dict(norm="const", steps=3, resolution=768, init_noise=_noise(2024, 28, 96))
    o32, usd, vsd, emb = build(UNetConfig(), MARIGOLD_V1, torch.float32, dev)
    d32, l32 = o32(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    del o32
    o16, *_ = build(UNetConfig(), MARIGOLD_V1, torch.bfloat16, dev)
    d16, l16 = o16(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    del o16
    torch.cuda.empty_cache()
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    torch.cuda.synchronize()
    assert dh.shape == (nb, 1, 352, 1216) and lh.shape == (nb, 4, 28, 96) and torch.isfinite(dh).all()
    worst = (0.0, 0.0)
    for i in range(nb):
        sl = slice(i, i + 1)
        mean_h, p99_h = fitted_error(dh[sl], d32[sl].cpu(), sparses[sl])
        mean_b, p99_b = fitted_error(d16[sl].cpu(), d32[sl].cpu(), sparses[sl])
        lat_h, lat_b = _lat_err(lh[sl], l32[sl]), _lat_err(l16[sl], l32[sl])
        print(f"\nC4 batch {nb} frame {i} (full UNet, 1216x352, 64-beam, 3 steps): HIP fitted |d| mean {mean_h:.5f} "
              f"p99 {p99_h:.5f} latent {lat_h:.4f} | oracle-bf16 mean {mean_b:.5f} p99 {p99_b:.5f} latent {lat_b:.4f}")
        worst = (max(worst[0], mean_h), max(worst[1], p99_h))
        assert mean_h <= 2 * mean_b + 2e-3 and p99_h <= 2 * p99_b + 2e-3
        assert lat_h <= 2 * lat_b + 2e-3
    print(f"C4 batch {nb} worst: mean {worst[0]:.5f} p99 {worst[1]:.5f}")
    assert worst[0] <= 0.02 and worst[1] <= 0.08


def test_c4_full_unet_50_steps():
    """C4 (KITTI 1216x352 at resolution 768, 64-beam LiDAR) through the FULL Marigold v1-0 UNet for the whole 50
    guided steps, one frame, against the fp32 oracle after the closed-form fit -- the C2 50-step test's bounds:
    2x the bf16 oracle's own drift + 1e-3 (fitted |d| mean / p99 of the depth range) and on the latent."""
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    imgs, sparses = _kitti_frames(1, seed=61)
    kw = dict(norm="const", steps=50, resolution=768, init_noise=_noise(2024, 28, 96))
    o32, usd, vsd, emb = build(UNetConfig(), MARIGOLD_V1, torch.float32, dev)
    d32, l32 = o32(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    del o32
    o16, *_ = build(UNetConfig(), MARIGOLD_V1, torch.bfloat16, dev)
    d16, l16 = o16(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    del o16
    torch.cuda.empty_cache()
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    dh, lh = pipe(imgs.to(dev), sparses.to(dev), 120.0, **kw)
    torch.cuda.synchronize()
    assert dh.shape == (1, 1, 352, 1216) and lh.shape == (1, 4, 28, 96) and torch.isfinite(dh).all()
    mean_h, p99_h = fitted_error(dh, d32.cpu(), sparses)
    mean_b, p99_b = fitted_error(d16.cpu(), d32.cpu(), sparses)
    lat_h, lat_b = _lat_err(lh, l32), _lat_err(l16, l32)
    print(f"\nC4 (full UNet, 1216x352, 64-beam, 50 steps): HIP fitted |d| mean {mean_h:.5f} p99 {p99_h:.5f} "
          f"latent {lat_h:.4f} | oracle-bf16 mean {mean_b:.5f} p99 {p99_b:.5f} latent {lat_b:.4f}")
    assert mean_h <= 2 * mean_b + 1e-3 and p99_h <= 2 * p99_b + 1e-3
    assert lat_h <= 2 * lat_b + 2e-3
    # absolute, as the C2 50-step test: measured HIP 2.46 % mean / 9.26 % p99 of the range against the bf16 oracle's
    # own 2.44 % / 9.18 % drift from fp32 (profiles/r05r/), ~40 % headroom
    assert mean_h <= 0.035 and p99_h <= 0.13


def test_c5_full_unet_ensemble_10_steps():
    """C5 (nuScenes 1600x900 at resolution 768: latent 54x96, 3000 points) with the 10-seed ensemble as ONE
    batch-10 call through the FULL Marigold v1-0 UNet, 10 guided steps, then mean + compute_affine_params
    (marigold_dc.py:53-128), against the oracle's per-seed loop.  Bound: 2x the bf16 oracle's own error + 2e-3
    of the range (mean |d|), and per seed the latent within 2x the bf16 oracle's latent error + 2e-3."""
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    h, w = 900, 1600
    imgs, sparses = synth_inputs(1, h, w, 3000, seed=50)
    seeds = list(range(2024, 2034))
    noises = [_noise(sd, 54, 96) for sd in seeds]
    kw = dict(norm="const", steps=10, resolution=768)
    lat32, lat16 = [], []
    o32, usd, vsd, emb = build(UNetConfig(), MARIGOLD_V1, torch.float32, dev)
    r32, *_ = P.ensemble(_LatCollect(o32, lat32), imgs.to(dev), sparses.to(dev), 120.0, noises, **kw)
    del o32
    o16, *_ = build(UNetConfig(), MARIGOLD_V1, torch.bfloat16, dev)
    r16, *_ = P.ensemble(_LatCollect(o16, lat16), imgs.to(dev), sparses.to(dev), 120.0, noises, **kw)
    del o16
    torch.cuda.empty_cache()
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    dh, aff, lat = pipe.ensemble(imgs.to(dev), sparses.to(dev), 120.0, seeds=seeds, **kw)
    torch.cuda.synchronize()
    assert dh.shape == (1, 1, h, w) and aff.shape == (1, 2) and lat.shape == (10, 4, 54, 96)
    assert torch.isfinite(dh).all()
    rng = float(r32.max() - r32.min())
    err_h = float((dh.cpu() - r32.cpu()).abs().mean()) / rng
    err_b = float((r16.cpu() - r32.cpu()).abs().mean()) / rng
    p99_h = float(torch.quantile(((dh.cpu() - r32.cpu()).abs() / rng).flatten()[::7], 0.99))
    lat_e = [(_lat_err(lat[k:k + 1], lat32[k]), _lat_err(lat16[k], lat32[k])) for k in range(10)]
    print(f"\nC5 10-seed ensemble (full UNet, 1600x900, 3000 pts, 10 steps): HIP |d| mean {err_h:.5f} p99 {p99_h:.5f} "
          f"of range | oracle-bf16 {err_b:.5f}; per-seed latent HIP/bf16 "
          + " ".join(f"{a:.4f}/{b:.4f}" for a, b in lat_e))
    assert err_h <= 2 * err_b + 2e-3
    for a, b in lat_e:
        assert a <= 2 * b + 2e-3


class _LatCollect:
    """Wraps an oracle pipeline: forwards calls, keeps each call's output latents (one per seed)."""

    def __init__(self, pipe, sink):
        self.pipe, self.sink = pipe, sink

    def __call__(self, *a, **k):
        d, lat = self.pipe(*a, **k)
        self.sink.append(lat.detach().cpu())
        return d, lat

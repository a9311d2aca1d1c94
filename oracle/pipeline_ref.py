"""CPU restatement of the Marigold-DC guided sampler (reference ``marigold_dc.py``).

TEST INFRASTRUCTURE ONLY -- the checker for the HIP path; never imported by
``depth_completion_amd``.

Every function cites the reference lines it restates.  The restatement keeps
the reference's operation order and dtype placement (bf16 latents/Adam state,
fp32 affine parameters and loss) so that, on the CPU, it reproduces the
reference's own code bit-for-bit; ``tests/test_oracle_golden.py`` checks that
against vectors produced by running the reference functions themselves
(``tests/golden/make_golden.py``).
"""
from __future__ import annotations

from contextlib import nullcontext

import torch
from torch.optim import SGD, Adagrad, Adam

from .diffusers_ref import MarigoldImageProcessor

EPSILON = 1e-7                                   # marigold_dc.py:20
SUPPORTED_LOSS_FUNCS = ["l1", "l2", "edge", "smooth"]   # marigold_dc.py:19


# ---------------------------------------------------------------- utils.py
def masked_minmax(x, mask, dim=None):
    """utils.py:89-138: min/max over masked entries; ValueError on an empty mask."""
    if x.shape != mask.shape:
        raise ValueError(f"Shape of x {x.shape} must be equal to shape of mask {mask.shape}")
    inf = torch.tensor(float("inf"), device=x.device, dtype=x.dtype)
    lo = torch.where(mask, x, inf)
    hi = torch.where(mask, x, -inf)
    if dim is None:
        mn, mx = lo.min(), hi.max()
    else:
        mn, mx = lo.amin(dim=dim), hi.amax(dim=dim)
    if torch.isinf(mn).any() or torch.isinf(mx).any():
        raise ValueError("No valid values found in mask for some positions.")
    return mn, mx


def kld_stdnorm(x, reduction="mean", mode="simple"):
    """utils.py:28-86."""
    n = x.shape[0]
    flat = x.reshape(n, -1)
    eps = torch.finfo(x.dtype).eps
    if mode == "simple":
        dist = flat.square().mean(dim=-1)
    elif mode == "strict":
        mu = flat.mean(dim=-1)
        var = flat.var(dim=-1, unbiased=False)
        dist = 0.5 * (mu.square() + var - torch.log(var + eps) - 1)
    else:
        raise ValueError(f"Unknown mode: {mode}")
    if reduction == "mean":
        return dist.mean()
    if reduction == "sum":
        return dist.sum()
    if reduction == "none":
        return dist
    raise ValueError(f"Unknown reduction: {reduction}")


# ---------------------------------------------------------- marigold_dc.py
def get_projection_fn(projection):
    """marigold_dc.py:23-50."""
    table = {"log": torch.log, "log10": torch.log10, "linear": lambda v: v}
    if projection not in table:
        raise ValueError(f"Unknown projection method: {projection}")
    return table[projection]


def compute_affine_params(affines, guides, masks):
    """marigold_dc.py:53-128: masked least-squares scale/shift per sample."""
    n = affines.shape[0]
    a = affines.view(n, -1)
    g = guides.view(n, -1)
    m = masks.view(n, -1)
    cnt = m.sum(dim=1, keepdim=True)
    if torch.any(cnt == 0):
        raise ValueError("At least one mask in the batch has no valid points")
    a_mean = torch.sum(a * m, dim=1, keepdim=True) / cnt
    g_mean = torch.sum(g * m, dim=1, keepdim=True) / cnt
    ac = (a - a_mean) * m
    gc = (g - g_mean) * m
    var = torch.sum(ac.pow(2), dim=1, keepdim=True)
    cov = torch.sum(ac * gc, dim=1, keepdim=True)
    scale = cov / (var + EPSILON)
    shift = g_mean - scale * a_mean
    return scale.squeeze(1), shift.squeeze(1)


def compute_loss(denses, sparses, masks, loss_funcs, images=None, kld=False,
                 kld_weight=0.1, kld_mode="simple", pred_latents=None):
    """marigold_dc.py:131-245 (l1/l2 on the hot path; edge/smooth/kld restated for completeness)."""
    if len(loss_funcs) == 0:
        raise ValueError("loss_funcs must contain at least one loss function")
    if kld and pred_latents is None:
        raise ValueError("pred_latents must be provided when kl-divergence constraint is enabled")
    total = torch.zeros(denses.shape[0], device=denses.device)
    for name in loss_funcs:
        if name == "l1":
            total += (torch.abs(denses - sparses) * masks).sum(dim=(1, 2, 3)) / masks.sum(dim=(1, 2, 3))
        elif name == "l2":
            total += (((denses - sparses) ** 2) * masks).sum(dim=(1, 2, 3)) / masks.sum(dim=(1, 2, 3))
        elif name == "edge":
            if images is None:
                raise ValueError("image must be provided for edge loss")
            c = images.shape[1]
            if c == 3:
                gray = 0.299 * images[:, 0:1] + 0.587 * images[:, 1:2] + 0.114 * images[:, 2:3]
            elif c == 1:
                gray = images
            else:
                raise ValueError(f"Image must have 1 or 3 channels, got {c}")
            gpx = torch.abs(denses[:, :, :, :-1] - denses[:, :, :, 1:])
            gpy = torch.abs(denses[:, :, :-1, :] - denses[:, :, 1:, :])
            ggx = torch.abs(gray[:, :, :, :-1] - gray[:, :, :, 1:])
            ggy = torch.abs(gray[:, :, :-1, :] - gray[:, :, 1:, :])
            total += torch.abs(gpx - ggx).mean(dim=(1, 2, 3)) + torch.abs(gpy - ggy).mean(dim=(1, 2, 3))
        elif name == "smooth":
            if images is None:
                raise ValueError("image must be provided for smooth loss")
            lh = torch.abs(denses[:, :, :-1, :] - denses[:, :, 1:, :]).mean(dim=(1, 2, 3))
            lw = torch.abs(denses[:, :, :, :-1] - denses[:, :, :, 1:]).mean(dim=(1, 2, 3))
            total += lh + lw
        else:
            raise ValueError(f"Unknown loss function: {name}")
    if kld:
        total += kld_weight * kld_stdnorm(pred_latents, reduction="none", mode=kld_mode)
    return total


class MarigoldBase:
    """The [D] ``MarigoldDepthPipeline`` pieces the reference inherits (diffusers 0.31.0)."""

    def __init__(self, unet, vae, scheduler, empty_text_embedding, dtype=torch.float32, device="cpu"):
        self.unet = unet
        self.vae = vae
        self.scheduler = scheduler
        self.image_processor = MarigoldImageProcessor()
        self.empty_text_embedding = empty_text_embedding.to(device=device, dtype=dtype)
        self.tokenizer = None
        self.text_encoder = None
        self.dtype = dtype
        self.device = torch.device(device)

    def prepare_latents(self, image, latents, generator, ensemble_size, batch_size):
        """[D] MarigoldDepthPipeline.prepare_latents: retrieve_latents -> ``.latent_dist.mode()`` (AutoencoderKL)
        or ``.latents`` (TAESD), times the VAE's scaling_factor (0.18215 / 1.0)."""
        def retrieve(out):
            return out.latent_dist.mode() if hasattr(out, "latent_dist") else out.latents
        enc = [retrieve(self.vae.encode(image[i:i + batch_size])) for i in range(0, image.shape[0], batch_size)]
        img_lat = torch.cat(enc, dim=0) * self.vae.scaling_factor
        img_lat = img_lat.repeat_interleave(ensemble_size, dim=0)
        pred = latents
        if pred is None:
            pred = torch.randn(img_lat.shape, generator=generator, device=img_lat.device,
                               dtype=img_lat.dtype)
        return img_lat, pred

    def decode_prediction(self, pred_latent):
        """[D] MarigoldDepthPipeline.decode_prediction."""
        pred = self.vae.decode(pred_latent / self.vae.scaling_factor, return_dict=False)[0]
        pred = pred.mean(dim=1, keepdim=True)
        pred = torch.clip(pred, -1.0, 1.0)
        return (pred + 1.0) / 2.0


class OracleMarigoldDC(MarigoldBase):
    """Restatement of ``MarigoldDepthCompletionPipeline`` (marigold_dc.py:248-985)."""

    def _affine_to_metric(self, affines, guides, masks, closed_form=False, affine_params=None):
        """marigold_dc.py:284-336."""
        if not closed_form and affine_params is None:
            raise ValueError("affine_params must be provided when closed_form is False")
        n = affines.shape[0]
        if not closed_form:
            s, sh = affine_params
            lo, hi = masked_minmax(guides.view(n, -1), masks.view(n, -1), dim=-1)
            lo = lo.view(n, 1, 1, 1)
            hi = hi.view(n, 1, 1, 1)
            return (s ** 2) * (hi - lo) * affines + (sh ** 2) * lo
        s, sh = compute_affine_params(affines, guides, masks)
        return s.view(n, 1, 1, 1) * affines + sh.view(n, 1, 1, 1)

    def _latent_to_affine(self, latents, orig_res, padding, interp_mode="bilinear"):
        """marigold_dc.py:338-371."""
        aff = self.decode_prediction(latents)
        aff = self.image_processor.unpad_image(aff, padding)
        return self.image_processor.resize_antialias(aff, orig_res, interp_mode)

    def _latent_to_metric(self, latents, guides, masks, orig_res, padding, affine_params=None,
                          closed_form=False, interp_mode="bilinear"):
        """marigold_dc.py:373-430."""
        aff = self._latent_to_affine(latents, orig_res, padding, interp_mode=interp_mode)
        return self._affine_to_metric(aff, guides, masks, closed_form=closed_form, affine_params=affine_params)

    def _predict_noise(self, img_latents, pred_latents, t):
        """marigold_dc.py:432-465."""
        n = img_latents.shape[0]
        x = torch.cat([img_latents, pred_latents], dim=1)
        return self.unet(x, t, encoder_hidden_states=self.empty_text_embedding.repeat(n, 1, 1),
                         return_dict=False)[0]

    @staticmethod
    def _depth_space(d, projection, inv, lo, hi, lo_p, hi_p):
        """marigold_dc.py:843-860 / 930-948 (non-linear projection or inverse)."""
        if projection != "linear":
            d = d * (hi - lo) + lo
            d = get_projection_fn(projection)(d)
            if inv:
                d = 1 / d
            return (d - lo_p) / (hi_p - lo_p)
        if inv:
            d = d * (hi - lo) + lo
            d = 1 / d
            return (d - lo_p) / (hi_p - lo_p)
        return d

    def __call__(self, imgs, sparses, max_depth, min_depth=0.0, projection="linear", inv=False,
                 norm="minmax", percentile=(0.01, 0.99), pred_latents_prev=None, beta=0.9, steps=50,
                 resolution=768, closed_form=None, opt="adam", lr=None, kld=False, kld_weight=0.1,
                 kld_mode="simple", interp_mode="bilinear", loss_funcs=None, seed=2024,
                 train_latents=True, train_method="per-step", train_steps=10, init_noise=None, step_hook=None):
        """marigold_dc.py:467-985.  ``init_noise`` (build extension) overrides the seeded draw; ``step_hook``
        (test infrastructure) observes / replays the guided loop per step (see the loop below)."""
        # --- validation (marigold_dc.py:583-656)
        if (imgs.ndim != 4 or sparses.ndim != 4 or imgs.shape[0] != sparses.shape[0]
                or imgs.shape[-2:] != sparses.shape[-2:]):
            raise ValueError("Shape of image must be [N, C, H, W] and shape of sparse must be "
                             f"[N, 1, H, W], but got image.shape: {imgs.shape} and sparse.shape: {sparses.shape}")
        n, _, h, w = imgs.shape
        eh = resolution * h // (8 * max(h, w))
        ew = resolution * w // (8 * max(h, w))
        if pred_latents_prev is not None and (pred_latents_prev.ndim != 4
                                              or pred_latents_prev.shape != (n, 4, eh, ew)):
            raise ValueError(f"Shape of pred_latents_prev must be [N, 4, EH, EW], but got {pred_latents_prev.shape}")
        if closed_form is None:
            closed_form = not train_latents
        elif not closed_form and not train_latents:
            raise ValueError("Closed form solution must be enabled when trainable latents are not used.")
        if train_method not in ["per-step", "per-input"]:
            raise ValueError(f"Unknown train_method: {train_method}")
        if train_method == "per-input" and train_steps <= 0:
            raise ValueError("train_steps must be > 0 when per-input training is enabled")
        if not (0 < beta < 1):
            raise ValueError(f"beta must be in (0, 1), but got {beta}")
        if norm == "percentile" and not all(0 <= p <= 1 for p in percentile):
            raise ValueError(f"percentile must be in [0, 1], but got {percentile}")
        if projection not in ["linear", "log", "log10"]:
            raise ValueError(f"Unknown projection method: {projection}")
        if (projection in ["log", "log10"] or inv) and min_depth <= EPSILON:
            raise ValueError(f"min_depth must be > {EPSILON} when projection is 'log' or 'log10' "
                             f"or inv is True, but got {min_depth}")
        lr_lat, lr_aff = (0.05, 0.005) if lr is None else lr
        if loss_funcs is None:
            loss_funcs = ["l1", "l2"]
        else:
            for f in loss_funcs:
                if f not in SUPPORTED_LOSS_FUNCS:
                    raise ValueError(f"Unknown loss function: {f}")

        # --- preprocessing (marigold_dc.py:658-756)
        with torch.no_grad():
            gen = torch.Generator(device=self.device).manual_seed(seed)
            if init_noise is None:
                common = torch.randn((1, 4, eh, ew), device=imgs.device, dtype=self.dtype, generator=gen)
            else:
                common = init_noise.to(device=imgs.device, dtype=self.dtype)
                torch.randn((1, 4, eh, ew), device=imgs.device, dtype=self.dtype, generator=gen)
            common = common.repeat(n, 1, 1, 1)
            x_img, padding, orig_res = self.image_processor.preprocess(
                imgs, processing_resolution=resolution, device=self.device, dtype=self.dtype)
            orig_res = tuple(orig_res)
            img_lat, _ = self.prepare_latents(x_img, None, gen, 1, n)
            if pred_latents_prev is not None:
                lat = beta * common + (1 - beta) * pred_latents_prev
            else:
                lat = common
            masks = sparses > 0
            if norm == "minmax":
                lo, hi = masked_minmax(sparses.view(n, -1), masks.view(n, -1), dim=-1)
                lo, hi = lo.view(n, 1, 1, 1), hi.view(n, 1, 1, 1)
            elif norm == "percentile":
                p = torch.tensor(percentile, device=sparses.device)
                r = torch.stack([torch.quantile(s[m], p) for s, m in zip(sparses, masks, strict=True)])
                lo, hi = r[:, 0].view(n, 1, 1, 1), r[:, 1].view(n, 1, 1, 1)
            elif norm == "const":
                lo = torch.full((n, 1, 1, 1), min_depth, device=sparses.device)
                hi = torch.full((n, 1, 1, 1), max_depth, device=sparses.device)
            else:
                raise ValueError(f"Unknown norm method: {norm}")
            sp_cl = sparses.clamp(min=lo, max=hi)
            if norm in ["minmax", "percentile"]:
                lo = lo.clamp(min=min_depth)
                hi = hi.clamp(max=max_depth)
            proj = get_projection_fn(projection)
            lo_p, hi_p, sp_p = proj(lo), proj(hi), proj(sp_cl)
            if inv:
                lo_p, hi_p = 1 / hi_p, 1 / lo_p
                sp_p = 1 / sp_p
            guides = (sp_p - lo_p) / (hi_p - lo_p)

        # --- trainables + optimizer (marigold_dc.py:758-789)
        per_step = train_latents and train_method == "per-step"
        if per_step:
            lat = torch.nn.Parameter(lat)
        aff_params = ((torch.nn.Parameter(torch.ones(n, 1, 1, 1, device=self.device)),
                       torch.nn.Parameter(torch.zeros(n, 1, 1, 1, device=self.device)))
                      if (not closed_form and train_latents) else None)
        optim = None
        if train_latents:
            groups = [{"params": [lat], "lr": lr_lat}]
            if aff_params is not None:
                groups.append({"params": list(aff_params), "lr": lr_aff})
            if opt == "adam":
                optim = Adam(groups)
            elif opt == "sgd":
                optim = SGD(groups)
            elif opt == "adagrad":
                optim = Adagrad(groups)
            else:
                raise ValueError(f"Unknown optimizer: {opt}")

        # --- denoising loop (marigold_dc.py:791-909)
        # step_hook (test infrastructure, not in the reference): step_hook("pre", i, t, state) before and
        # step_hook("post", i, t, state) after each guided step; state = {"lat", "img_lat", "optim", "aff"} (+ "v",
        # "grad" -- lat.grad after the rescale -- at "post").  A "pre" hook may overwrite lat.data, the optimiser
        # state or state["img_lat"] in place: the per-step (teacher-forced) parity test replays another
        # execution's trajectory one step at a time this way.
        guided_hook = step_hook if (optim is not None and train_method == "per-step") else None
        with (nullcontext() if per_step else torch.no_grad()):
            self.scheduler.set_timesteps(steps, device=self.device)
            for i, t in enumerate(self.scheduler.timesteps):
                if guided_hook is not None:
                    state = {"lat": lat, "img_lat": img_lat, "optim": optim, "aff": aff_params}
                    guided_hook("pre", i, t, state)
                    img_lat = state["img_lat"]
                if optim is not None and train_method == "per-step":
                    optim.zero_grad()
                v = self._predict_noise(img_lat, lat, t)
                if optim is not None and train_method == "per-step":
                    with torch.no_grad():
                        a_t = self.scheduler.alphas_cumprod[t]
                        b_t = 1 - a_t
                        eps = (a_t ** 0.5) * v + (b_t ** 0.5) * lat
                    x0 = self.scheduler.step(v, t, lat, generator=gen).pred_original_sample
                    d = self._latent_to_metric(x0, guides, masks, orig_res, padding, affine_params=aff_params,
                                               closed_form=closed_form, interp_mode=interp_mode).clamp(0.0, 1.0)
                    d = self._depth_space(d, projection, inv, lo, hi, lo_p, hi_p)
                    losses = compute_loss(d, guides, masks, loss_funcs, images=imgs, kld=kld,
                                          kld_weight=kld_weight, kld_mode=kld_mode, pred_latents=lat)
                    losses.backward(torch.ones_like(losses))
                    with torch.no_grad():
                        en = torch.linalg.norm(eps.view(n, -1), dim=1)
                        gn = torch.linalg.norm(lat.grad.view(n, -1), dim=1)
                        lat.grad *= (en / gn.clamp(min=EPSILON)).view(n, 1, 1, 1)
                    optim.step()
                    with torch.no_grad():
                        lat.data = self.scheduler.step(v, t, lat, generator=gen).prev_sample
                    if guided_hook is not None:
                        state.update(v=v.detach(), grad=lat.grad.detach())
                        guided_hook("post", i, t, state)
                else:
                    lat = self.scheduler.step(v, t, lat, generator=gen).prev_sample

        # --- per-input training (marigold_dc.py:911-967)
        if optim is not None and train_method == "per-input":
            lat = torch.nn.Parameter(lat)
            # NOTE: the reference's optimizer still holds the pre-loop tensor (marigold_dc.py:777-783);
            # restated as-is.
            for _ in range(train_steps):
                optim.zero_grad()
                d = self._latent_to_metric(lat, guides, masks, orig_res, padding, affine_params=aff_params,
                                           closed_form=closed_form, interp_mode=interp_mode)
                d = self._depth_space(d, projection, inv, lo, hi, lo_p, hi_p)
                losses = compute_loss(d, guides, masks, loss_funcs, images=imgs, kld=kld,
                                      kld_weight=kld_weight, kld_mode=kld_mode, pred_latents=lat)
                losses.backward(torch.ones_like(losses))
                optim.step()

        # --- final decode (marigold_dc.py:969-985)
        with torch.no_grad():
            out_lat = lat.detach()
            d = self._latent_to_metric(out_lat, guides, masks, orig_res, padding, affine_params=aff_params,
                                       closed_form=closed_form, interp_mode=interp_mode).clamp(0.0, 1.0)
            dense = d * (hi - lo) + lo
        return dense, out_lat


# ------------------------------------------------- seed ensemble (BASELINE.json config C5)
def ensemble(pipe, imgs, sparses, max_depth, noises, **kw):
    """C5's per-frame seed ensemble: one reference call per seed (initial noise ``noises[k]`` [1, 4, h, w]),
    the mean of the dense maps over the seeds (torch.stack(...).mean(0)), then compute_affine_params
    (marigold_dc.py:53-128) of the mean against the sparse depth over sparses > 0, applied.
    Returns (fitted dense [N, 1, H, W], scale [N], shift [N])."""
    denses = [pipe(imgs, sparses, max_depth, init_noise=nz, **kw)[0].float() for nz in noises]
    mean = torch.stack(denses).mean(0)
    scale, shift = compute_affine_params(mean, sparses.float(), sparses > 0)
    return mean * scale.view(-1, 1, 1, 1) + shift.view(-1, 1, 1, 1), scale, shift

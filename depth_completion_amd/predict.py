"""predict.py-compatible command line for the MI355X sampler (predict.py:25-781).

    python -m depth_completion_amd.predict SRC_ROOT DST_ROOT [options]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m depth_completion_amd.predict SRC_ROOT DST_ROOT [options]      # frames sharded per GPU

Same arguments, defaults and coercions as the reference CLI (predict.py:25-457); the differences:
* weights load from a local diffusers-format directory (``--weights DIR`` with ``unet/`` and
  ``taesd/`` safetensors plus ``empty_text_embedding.safetensors``) instead of the hub, or from
  seeded synthetic weights (``--synthetic-weights SEED``) -- there is no network;
* ``--model lcm`` and ``--precision fp32`` are rows the HIP path does not run yet and fail loudly
  (``--vae original`` runs the AutoencoderKL of depth_completion_amd/vae_kl.py); ``--compile-graph`` / ``--compile-mode`` are accepted and ignored (the step is
  always a captured hipGraph);
* under torch.distributed.run each rank processes a contiguous shard of every dataset's frames
  (depth_completion_amd/shard.py); ``--use-prev-latent`` chains stay inside a shard.
"""
from __future__ import annotations

import logging
import os
import sys
import time
from pathlib import Path

import click
import torch

from . import io as dio
from .shard import frame_shard

logger = logging.getLogger("depth_completion_amd.predict")
SUPPORTED_LOSS_FUNCS = ["l1", "l2", "edge", "smooth"]   # marigold_dc.py:19


class CommaSeparated(click.ParamType):
    """utils.py:742-814: comma-separated values of one type."""
    name = "comma_separated"

    def __init__(self, typ):
        self.typ = typ

    def convert(self, value, param, ctx):
        if isinstance(value, (list, tuple)):
            return list(value)
        try:
            return [self.typ(v.strip()) for v in str(value).split(",") if v.strip()]
        except ValueError:
            self.fail(f"{value!r} is not a comma-separated list of {self.typ.__name__}", param, ctx)


def load_weights(weights: Path | None, synthetic_seed: int | None, unet_config: str, vae: str = "light"):
    """(unet state, VAE state, empty-prompt embedding, UNet config, VAE config): the light VAE is TAESD
    (``taesd/``), the original one the Marigold checkpoint's AutoencoderKL (``vae/``)."""
    from . import synthetic
    from .config import MARIGOLD_V1, TINY
    from .vae_kl import SD_VAE, TINY_KL
    cfg = TINY if unet_config == "tiny" else MARIGOLD_V1
    kcfg = TINY_KL if unet_config == "tiny" else SD_VAE
    if weights is not None:
        from safetensors.torch import load_file
        unet = load_file(str(weights / "unet" / "diffusion_pytorch_model.safetensors"))
        sub = "taesd" if vae == "light" else "vae"
        vsd = load_file(str(weights / sub / "diffusion_pytorch_model.safetensors"))
        emb = load_file(str(weights / "empty_text_embedding.safetensors"))["embedding"]
        return unet, vsd, emb, cfg, kcfg
    seed = 0 if synthetic_seed is None else synthetic_seed
    vsd = synthetic.taesd_state_dict(seed + 12) if vae == "light" else synthetic.kl_state_dict(kcfg, seed + 12)
    return (synthetic.unet_state_dict(cfg, seed + 11), vsd, synthetic.text_embedding(seed + 13, cfg.cross_attention_dim),
            cfg, kcfg)


def discover(src_root: Path, use_segmask: bool):
    """predict.py:514-580: datasets -> paired (image, sparse[, segmask]) paths."""
    datasets = dio.find_dataset_dirs(src_root)
    plan = []
    for d in datasets:
        seg_ok = use_segmask
        segdir = d / dio.DATASET_DIR_NAME_SEGMASK
        segmap = None
        if not segdir.exists():
            if use_segmask:
                logger.error(f"No segmentation directory found at {segdir}. Segmentation masks will not used for {d.name}")
            seg_ok = False
        elif not (segdir / "map.csv").exists():
            if use_segmask:
                logger.error(f"No segmentation mapping file found at {segdir / 'map.csv'}")
            seg_ok = False
        else:
            segmap = dio.load_segmap(segdir / "map.csv")
        img_dir, sp_dir = d / dio.DATASET_DIR_NAME_IMAGE, d / dio.DATASET_DIR_NAME_SPARSE
        pairs = []
        for p in sorted(dio.find_img_paths(img_dir), key=lambda x: x.name):
            sp = sp_dir / p.relative_to(img_dir).with_suffix(".png")
            if not sp.exists():
                logger.warning(f"No sparse depth map found for image {p} (skipped)")
                continue
            sm = segdir / p.relative_to(img_dir).with_suffix(".png")
            if seg_ok and not sm.exists():
                logger.warning(f"No segmentation mask found for image {p} (skipped)")
                continue
            pairs.append((p, sp, sm if seg_ok else None))
        plan.append((d, pairs, segmap if seg_ok else None))
    return plan


def frame_outputs(out_dir: Path, img_dir: Path, sp_dir: Path, ip: Path, sp: Path, compress: str, save_dense: bool,
                  vis: bool) -> list:
    """The files one input pair writes (dense map and/or visualisation), as the loop below names them."""
    outs = []
    if save_dense:
        outs.append((out_dir / dio.RESULT_DIR_NAME_DENSE / sp.relative_to(sp_dir)).parent
                    / sp.with_suffix(f".{compress}").name)
    if vis:
        outs.append((out_dir / dio.RESULT_DIR_NAME_VIS / ip.relative_to(img_dir)).parent / f"{ip.stem}_vis.jpg")
    return outs


def pending_pairs(pairs: list, out_dir: Path, img_dir: Path, sp_dir: Path, compress: str, save_dense: bool,
                  vis: bool) -> list:
    """--resume: drop the pairs whose every output already exists (SURVEY.md §5 'checkpoint / resume'; the
    reference has none and re-runs overwrite).  A pair with any output missing is re-run in full."""
    keep = []
    for ip, sp, sm in pairs:
        outs = frame_outputs(out_dir, img_dir, sp_dir, ip, sp, compress, save_dense, vis)
        if not outs or not all(o.exists() for o in outs):
            keep.append((ip, sp, sm))
    return keep


@click.command(help="Predict dense depth maps from sparse depth maps and camera images (MI355X).")
@click.argument("src_root", type=click.Path(exists=True, path_type=Path, file_okay=False, dir_okay=True))
@click.argument("dst_root", type=click.Path(exists=False, path_type=Path))
@click.option("--model", type=click.Choice(["original", "lcm"]), default="original", show_default=True)
@click.option("--vae", type=click.Choice(["original", "light"]), default="light", show_default=True)
@click.option("-n", "--steps", type=click.IntRange(min=1), default=50, show_default=True)
@click.option("-r", "--res", type=click.IntRange(min=1), default=768, show_default=True)
@click.option("--norm", type=click.Choice(["const", "minmax", "percentile"]), default="const", show_default=True)
@click.option("--percentile", type=CommaSeparated(float), default="0.01,0.99", show_default=True)
@click.option("--max-sparse-depth", type=click.FloatRange(min=0, min_open=True), default=120.0, show_default=True)
@click.option("--max-depth", type=click.FloatRange(min=0, min_open=True), default=120.0, show_default=True)
@click.option("--min-depth", type=click.FloatRange(min=0), default=0.0, show_default=True)
@click.option("-v", "--vis", type=bool, default=True, show_default=True)
@click.option("-vr", "--vis-res", type=click.Tuple([int, int]), default=(512, -1), show_default=True)
@click.option("-vo", "--vis-order", type=CommaSeparated(str), default="image,sparse,dense", show_default=True)
@click.option("--save-dense", type=bool, default=True, show_default=True)
@click.option("--log", type=click.Path(path_type=Path), default=None, show_default=True)
@click.option("--log-level", type=click.Choice(["TRACE", "DEBUG", "INFO", "SUCCESS", "WARNING", "ERROR", "CRITICAL"]),
              default="INFO", show_default=True)
@click.option("-p", "--precision", type=click.Choice(["bf16", "fp32"]), default="bf16", show_default=True)
@click.option("-c", "--compress", type=click.Choice(["npz", "bl2", "npy"]), default="bl2", show_default=True)
@click.option("--compile-graph", type=bool, default=False, show_default=True)
@click.option("--compile-mode", type=click.Choice(["max-autotune", "reduce-overhead", "default"]),
              default="reduce-overhead", show_default=True)
@click.option("--interp-mode", type=click.Choice(["bilinear", "nearest"]), default="bilinear", show_default=True)
@click.option("--loss-funcs", type=CommaSeparated(str), default="l1,l2", show_default=True)
@click.option("--opt", type=click.Choice(["adam", "sgd", "adagrad"]), default="adam", show_default=True)
@click.option("--lr-latent", type=click.FloatRange(min=0, min_open=True), default=0.05, show_default=True)
@click.option("--lr-scaling", type=click.FloatRange(min=0, min_open=True), default=0.005, show_default=True)
@click.option("--kld", type=bool, default=False, show_default=True)
@click.option("--kld-mode", type=click.Choice(["simple", "strict"]), default="simple", show_default=True)
@click.option("--kld-weight", type=click.FloatRange(min=0, min_open=True), default=0.1, show_default=True)
@click.option("-bs", "--batch-size", type=click.IntRange(min=1), default=1, show_default=True)
@click.option("--use-prev-latent", type=bool, default=False, show_default=True)
@click.option("--beta", type=click.FloatRange(min=0, min_open=True), default=0.9, show_default=True)
@click.option("--use-segmask", type=bool, default=False, show_default=True)
@click.option("--closed-form", type=bool, default=False, show_default=True)
@click.option("--projection", type=click.Choice(["linear", "log", "log10"]), default="linear", show_default=True)
@click.option("--inv", type=bool, default=False, show_default=True)
@click.option("--train-latents", type=bool, default=True, show_default=True)
@click.option("--train-method", type=click.Choice(["per-step", "per-input"]), default="per-step", show_default=True)
@click.option("--train-steps", type=click.IntRange(min=1), default=10, show_default=True)
@click.option("--weights", type=click.Path(exists=True, path_type=Path, file_okay=False), default=None,
              help="Local diffusers-format weights: unet/, taesd/, empty_text_embedding.safetensors.")
@click.option("--synthetic-weights", type=int, default=None, help="Seeded synthetic weights (no checkpoint).")
@click.option("--unet-config", type=click.Choice(["marigold-v1", "tiny"]), default="marigold-v1", hidden=True)
@click.option("--dry-run", is_flag=True, help="Discover and list the input pairs, run nothing.")
@click.option("--resume", is_flag=True, help="Skip input pairs whose outputs already exist (default: overwrite, as "
              "the reference does). With --use-prev-latent the warm-start chain restarts at the first pending frame.")
def main(src_root, dst_root, model, vae, steps, res, norm, percentile, max_sparse_depth, max_depth, min_depth, vis,
         vis_res, vis_order, save_dense, log, log_level, precision, compress, compile_graph, compile_mode,
         interp_mode, loss_funcs, opt, lr_latent, lr_scaling, kld, kld_mode, kld_weight, batch_size,
         use_prev_latent, beta, use_segmask, closed_form, projection, inv, train_latents, train_method, train_steps,
         weights, synthetic_weights, unet_config, dry_run, resume):
    level = {"TRACE": "DEBUG", "SUCCESS": "INFO"}.get(log_level, log_level)
    logging.basicConfig(level=getattr(logging, level), format="%(asctime)s %(levelname)s %(message)s",
                        stream=sys.stderr)
    if log is not None:
        log.parent.mkdir(parents=True, exist_ok=True)
        logging.getLogger().addHandler(logging.FileHandler(log))

    # ---- argument coercions (predict.py:400-457)
    if vis:
        vo = [v for v in vis_order if v in ("image", "sparse", "dense")]
        for v in vis_order:
            if v not in ("image", "sparse", "dense"):
                logger.error(f"Invalid order (skipped): {v}")
        if not vo:
            logger.critical("No valid visualization order specified")
            sys.exit(1)
        vis_order = vo
    lf = []
    for f in loss_funcs:
        if f not in SUPPORTED_LOSS_FUNCS:
            logger.error(f"Invalid loss function (skipped): {f}")
        else:
            lf.append(f)
    loss_funcs = lf
    if use_prev_latent and batch_size > 1:
        logger.warning("Currently, batch_size is forced to 1 when use_prev_latent=True.")
        batch_size = 1
    if (projection in ["log", "log10"] or inv) and norm == "const":
        logger.error("norm=const is not allowed when projection=log or log10. Falling back to norm=minmax")
        norm = "minmax"
    if model == "lcm" and train_latents:
        logger.error("LCM-based Marigold model does not support trainable latents. Falling back to train_latents=False")
        train_latents = False
    if not train_latents and not closed_form:
        logger.error("When trainable latentes are not used, closed-form solution must be enabled. "
                  "Falling back to closed_form=True")
        closed_form = True
    if compress == "bl2":
        try:
            import blosc2  # noqa: F401
        except ImportError:
            logger.error("compress=bl2 needs blosc2, which is not installed. Falling back to compress=npz")
            compress = "npz"

    plan = discover(src_root, use_segmask)
    if not plan:
        logger.critical(f"No dataset directories found at {src_root}")
        sys.exit(1)
    for d, pairs, _ in plan:
        if not pairs:
            logger.critical("No valid input pairs found")
            sys.exit(1)
        logger.info(f"Found {len(pairs):,} input pairs for {d.name}")
    if dry_run:
        for d, pairs, _ in plan:
            for p, sp, _ in pairs:
                print(f"{d.name}\t{p}\t{sp}")
        return

    # ---- rows the HIP path does not run (fail loudly, never approximate)
    if model == "lcm":
        raise click.UsageError("--model lcm (LCMScheduler) is not implemented on the MI355X path")
    if precision == "fp32":
        raise click.UsageError("--precision fp32 is not supported: the MI355X kernels compute in bf16")
    if compile_graph:
        logger.warning("--compile-graph is ignored: every guided step already runs as a captured hipGraph")
    if weights is None and synthetic_weights is None:
        raise click.UsageError("pass --weights DIR (local diffusers-format weights) or --synthetic-weights SEED")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        logger.critical("A GPU must be available to run this script.")
        sys.exit(1)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from .pipeline import MarigoldDepthCompletionPipeline
    usd, vsd, emb, cfg, kcfg = load_weights(weights, synthetic_weights, unet_config, vae)
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=cfg, device=dev, vae=vae, vae_config=kcfg)
    dst_root.mkdir(parents=True, exist_ok=True)

    for d, pairs, segmap in plan:
        out_dir = dst_root / d.relative_to(src_root)
        img_dir, sp_dir = d / dio.DATASET_DIR_NAME_IMAGE, d / dio.DATASET_DIR_NAME_SPARSE
        mine = [pairs[i] for i in frame_shard(len(pairs), rank, world)]
        if resume:
            n_all = len(mine)
            mine = pending_pairs(mine, out_dir, img_dir, sp_dir, compress, save_dense, vis)
            logger.info(f"--resume: {n_all - len(mine)} of {n_all} frames already done on rank {rank}")
        prev = None
        t0 = time.time()
        for b in range(0, len(mine), batch_size):
            batch = mine[b:b + batch_size]
            imgs_l = dio.load_img_tensors([p for p, _, _ in batch], "RGB", len(batch))
            sps_l = dio.load_img_tensors([s for _, s, _ in batch], "RGB", len(batch))
            flags = [i is not None and s is not None for i, s in zip(imgs_l, sps_l)]
            if not any(flags):
                logger.error(f"All images in batch {b + 1} failed to load (skipped)")
                continue
            batch = dio.filterout(batch, flags)
            imgs = torch.stack(dio.filterout(imgs_l, flags)).to(dev)
            sps = dio.to_depth(torch.stack(dio.filterout(sps_l, flags)).to(dev), max_distance=max_sparse_depth)
            denses, lat = pipe(imgs, sps, max_depth, min_depth=min_depth, projection=projection, inv=inv,
                               norm=norm, percentile=percentile, pred_latents_prev=prev, beta=beta, steps=steps,
                               resolution=res, interp_mode=interp_mode, loss_funcs=loss_funcs, opt=opt,
                               lr=(lr_latent, lr_scaling), kld=kld, kld_mode=kld_mode, kld_weight=kld_weight,
                               closed_form=closed_form, train_latents=train_latents, train_method=train_method,
                               train_steps=train_steps)
            if use_prev_latent:
                prev = lat
            for dense, sparse, img, (ip, sp, _) in zip(denses, sps, imgs, batch):
                if dio.has_nan(dense):
                    logger.error("NaN values found in dense depth map (skipped)")
                    continue
                outs = frame_outputs(out_dir, img_dir, sp_dir, ip, sp, compress, save_dense, vis)
                if save_dense:
                    dio.save_tensor(dense, outs[0], compress=compress)
                if vis:
                    mask = (sparse <= 0.0).repeat(img.shape[0], 1, 1).cpu()
                    views = []
                    for o in vis_order:
                        if o == "image":
                            views.append(img.cpu())
                        elif o == "sparse":
                            v = dio.visualize_depth(sparse[None].cpu(), max_depth=max_depth, min_depth=min_depth)[0]
                            v[mask] = 0
                            views.append(v)
                        else:
                            views.append(dio.visualize_depth(dense[None].cpu(), max_depth=max_depth,
                                                             min_depth=min_depth)[0])
                    grid = dio.make_grid(views, resize=tuple(vis_res))
                    dio.save_img_tensor(grid, outs[-1])
        logger.info(f"Finished processing {d.name} (rank {rank}/{world}: {len(mine)} frames, {time.time() - t0:.1f}s)")
    logger.info(f"Finished processing all {len(plan):,} datasets")


if __name__ == "__main__":
    main()

"""Benchmark: dense-depth frames/sec at 768x576 with 50 guided DDIM steps (BASELINE.json metric).

One bench "step" = one ``MarigoldDepthCompletionPipeline.__call__`` on one batch of synthetic
frames (default: config C2 = one 768x576 frame, 500 sparse points, 50 guided steps, bf16).
Multi-GPU: one process per GPU (torch.distributed.run), frames sharded across ranks with no
data-path collective (scaling = weak); the barrier + max-over-ranks timing is the only exchange.

Also reported on the same JSON line:
  roofline      the dominant kernel (implicit-GEMM conv/linear, dc_conv_gemm): the time a graph-replayed
                guided step spends in its conv launches (HIP events on the launch stream: the step's
                graph minus the same graph without them), algorithmic FLOPs / avg duration; `traffic`
                from the committed PMC pass
                (profiles/pmc_conv_gemm.json, FETCH_SIZE x2 + WRITE_SIZE per launch, gfx950 correction)
  cpu_baseline  the oracle (CPU PyTorch restatement of the reference path, incl. weight-gradients as
                the reference computes them) on this host's cores, rank 0 / N=1 only, on a bounded
                sample (1- and 2-step calls, extrapolated to 50 steps)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md "Peak BF16/FP16 MFMA")
PEAK_HBM_GBS = 8000.0


def synth_frame(h, w, n_points, seed):
    """Seeded RGB (smooth gradient + noise) + 8-bit quantised sparse depth."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, h), torch.linspace(0, 1, w), indexing="ij")
    img = (torch.stack([xx, yy, 0.5 * (xx + yy)]) * 200 + torch.randn((3, h, w), generator=g) * 12)
    img = img.clamp(0, 255).round().to(torch.uint8)
    field = 10 + 80 * yy + 20 * torch.sin(6.28 * xx + seed)
    k = (field * 255 / 120).round().clamp(1, 255)
    sp = torch.zeros(h * w)
    idx = torch.randperm(h * w, generator=g)[:n_points]
    sp[idx] = 120 * k.view(-1)[idx] / 255
    return img, sp.view(1, h, w)


def workload_name(h: int, w: int, batch: int) -> str:
    """BASELINE.json configs: C2 / C3 (768x576, 1 / 8 frames), C4 (KITTI 1216x352), C5 (nuScenes 1600x900,
    one seed of the ensemble); anything else is a custom shape."""
    if (h, w) == (576, 768):
        return "C2" if batch == 1 else "C3" if batch == 8 else f"C2-batch{batch}"
    return {(352, 1216): "C4", (900, 1600): "C5 (single seed)"}.get((h, w), "custom")


def conv_flops(d) -> float:
    """Algorithmic FLOPs of one dc_conv_gemm launch (real channels, valid taps only; a row-list launch
    counts its rows, padding included)."""
    M = d.nrows if d.rows else d.nb * d.hout * d.wout
    K = d.kh * d.kw * d.cin
    f = 2.0 * M * d.cout * K
    if d.mode == 2:   # transposed stride-2 gather: on average 1/4 of the taps are valid
        f /= 4.0
    return f


def measure_conv_kernel(pipe, st, reps: int = 3):
    """Time of the dominant kernel (dc_conv_gemm) inside one graph-replayed guided step.

    The step is captured twice as a hipGraph: as the timed region runs it, and with every
    dc_conv_gemm launch left out.  Each graph is replayed `reps` times between HIP events on the
    launch stream; the difference is the time the step spends in its conv launches, in the step's
    own order and cache state (no per-launch event packets).  Returns (launches, conv ms per step,
    algorithmic FLOPs per step).
    """
    from depth_completion_amd import ops
    from depth_completion_amd._lib import ConvDesc
    descs = []
    orig = ops.call

    def record(name, *args):
        if name == "dc_conv_gemm":
            descs.append(ConvDesc.from_buffer_copy(args[0]._obj))
        return orig(name, *args)

    def skip_conv(name, *args):
        return None if name == "dc_conv_gemm" else orig(name, *args)

    def timed_graph(hook):
        g = torch.cuda.CUDAGraph()
        ops.call = hook
        try:
            with torch.cuda.graph(g):
                pipe._step(st)
        finally:
            ops.call = orig
        stream = torch.cuda.current_stream()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            g.replay()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    torch.cuda.synchronize()
    st["dec"].set_rows(st.get("row_sets"))   # the timed calls' decode row lists (sparse-aware decode)
    try:
        t_all = timed_graph(record)
        n = len(descs)
        t_rest = timed_graph(skip_conv)
    finally:
        st["dec"].set_rows(None)
    flops = sum(conv_flops(d) for d in descs)
    return n, max(t_all - t_rest, 1e-6), flops


def cpu_baseline(h, w, n_points):
    """Oracle (CPU restatement) timed on this host: 1- and 2-step calls, extrapolated to 50 steps."""
    from oracle import pipeline_ref as P
    from oracle.diffusers_ref import (AutoencoderTiny, DDIMScheduler, UNet2DConditionModel, synthetic_state_dict,
                                      synthetic_taesd_state_dict, synthetic_text_embedding)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    unet = UNet2DConditionModel()
    unet.load_state_dict(synthetic_state_dict(unet, 11))
    vae = AutoencoderTiny()
    vae.load_state_dict(synthetic_taesd_state_dict(vae, 12))
    pipe = P.OracleMarigoldDC(unet.to(torch.bfloat16), vae.to(torch.bfloat16), DDIMScheduler(),
                              synthetic_text_embedding(13, 1024), dtype=torch.bfloat16)
    img, sp = synth_frame(h, w, n_points, 0)
    times = {}
    for s in (1, 2):
        t0 = time.perf_counter()
        pipe(img[None], sp[None], 120.0, norm="const", steps=s, resolution=768)
        times[s] = time.perf_counter() - t0
    t_step = max(times[2] - times[1], 1e-3)
    t_fixed = max(times[1] - t_step, 0.0)
    t_frame = t_fixed + 50 * t_step
    return {"value": 1.0 / t_frame, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"oracle bf16 CPU pipeline, 1 frame {w}x{h}, 1- and 2-step calls "
                      f"({times[1]:.1f}s, {times[2]:.1f}s) extrapolated to 50 guided steps "
                      f"({t_step:.2f} s/step incl. weight-grads)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="frames per call per GPU (C2: 1, C3: 8)")
    ap.add_argument("--height", type=int, default=576)
    ap.add_argument("--width", type=int, default=768)
    ap.add_argument("--points", type=int, default=500)
    ap.add_argument("--denoise-steps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from depth_completion_amd import synthetic
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    from depth_completion_amd.shard import frame_shard, max_over_ranks

    pipe = MarigoldDepthCompletionPipeline(synthetic.unet_state_dict(MARIGOLD_V1, 11), synthetic.taesd_state_dict(12),
                                           synthetic.text_embedding(13, 1024), device=dev,
                                           use_graph=not args.no_graph)
    B, H, W = args.batch, args.height, args.width
    # the job's frames 0..world*B-1, contiguous shard per rank (depth_completion_amd/shard.py)
    frames = [synth_frame(H, W, args.points, seed=i) for i in frame_shard(world * B, rank, world)]
    imgs = torch.stack([f[0] for f in frames]).to(dev)
    sps = torch.stack([f[1] for f in frames]).to(dev)
    kw = dict(norm="const", steps=args.denoise_steps, resolution=768)

    for _ in range(args.warmup):
        pipe(imgs, sps, 120.0, **kw)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dense, lat = pipe(imgs, sps, 120.0, **kw)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, device=dev)
    assert torch.isfinite(dense).all(), "non-finite dense output"

    frames_total = world * args.steps * B
    value = frames_total / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # dominant kernel roofline (rank 0 measures its own launches)
    st = pipe._plans[(B, pipe._call_state["h"], pipe._call_state["w"])]
    n_launch, conv_ms, conv_flops_ = measure_conv_kernel(pipe, st)
    avg_ms = conv_ms / max(n_launch, 1)
    achieved = conv_flops_ / (conv_ms * 1e-3) / 1e12
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_conv_gemm.json")
    if os.path.exists(pmc):   # committed PMC pass (tools/pmc_traffic.py), reported only for its own shape
        with open(pmc) as f:
            rec = json.load(f)
        if rec.get("latent_shape") == [B, pipe._call_state["h"], pipe._call_state["w"]]:
            traffic = round(rec["traffic_bytes_per_launch"])
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, C2 step)",
                "kernel": "dc_conv_gemm = conv_gemm_kernel (split-K partials reduced in-kernel by the last block), implicit-GEMM conv/linear",
                "launches_per_step": n_launch, "avg_launch_ms": round(avg_ms, 5),
                "method": "graph-replayed step minus the same graph without its conv launches (HIP events)",
                "algorithmic_gflop_per_step": round(conv_flops_ / 1e9, 1)}
    # whole-frame roofline: SURVEY §8(d) canonical 190.4 TFLOP per 768x576 frame (50 guided steps)
    frame_tflop = 190.4 * (args.denoise_steps / 50.0)
    step_roof = {"algorithmic_tflop_per_frame": frame_tflop,
                 "achieved_tflops_per_gpu": round(value / world * frame_tflop, 2),
                 "frac_of_bf16_peak": round(value / world * frame_tflop / PEAK_BF16_TFLOPS, 4),
                 "ceiling_fps_per_gpu": round(PEAK_BF16_TFLOPS / frame_tflop, 2)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(H, W, args.points)

    if rank == 0:
        line = {
            "metric": "dense-depth frames/sec at 768x576, 50 guided steps; 1 & 8 MI355X",
            "value": round(value, 4), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"{workload_name(H, W, B)}: {W}x{H} RGB + {args.points}-pt sparse depth, "
                                   f"{args.denoise_steps} guided DDIM steps, {B} frame(s) per call per GPU",
                       "frames_per_step": B * world, "resolution": 768, "guided_steps": args.denoise_steps,
                       "parallelism": f"frame-sharded dp{world} (no collectives)",
                       "weights": "synthetic seeded (Marigold v1-0 UNet + TAESD shapes)",
                       "hip_graph": not args.no_graph},
            "roofline": roofline, "frame_roofline": step_roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

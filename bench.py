"""Benchmark: dense-depth frames/sec at 768x576 with 50 guided DDIM steps (BASELINE.json metric).

One bench "step" = one ``MarigoldDepthCompletionPipeline.__call__`` (``ms_per_step``: one call) on one
batch of synthetic frames; default workload = config C2 (one 768x576 frame, 500 sparse points, 50
guided steps, bf16).  Every timed call gets FRESH frames (distinct seeds, same point count), so a
recapture of the step graph or new decode row lists fall inside the timed region; inputs are resident
in HBM before the clock starts.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) this process is one rank;
with ``--gpus N > 1`` and no WORLD_SIZE it spawns the N rank processes itself (before touching the GPU;
each child is a fresh interpreter, nothing re-execs) and exits with the first non-zero child status.
Frames shard across ranks with no data-path collective (scaling = weak); the barrier + max-over-ranks
timing is the only exchange.

Also reported on the JSON line:
  roofline       the dominant kernel (implicit-GEMM conv/linear, dc_conv_gemm): the time a graph-replayed
                 guided step spends in its conv launches (HIP events on the launch stream: the step's graph
                 minus the same graph without them), algorithmic FLOPs / that time; `traffic` / `hbm_gbs`
                 from the committed PMC passes over the graph-replayed step (profiles/pmc_step*.json, gfx950
                 corrections of MI355X_MICROARCH.md) for the latent shape they ran on;
                 `traffic_over_algorithmic` = those bytes over the launches' operands moved once (conv_bytes);
                 `mfma_util` = the PMC MFMA-busy cycles over the graph-timed family time x 2.4 GHz x 1024 SIMDs,
                 reported only when the record's conv_family_hash is this tree's (`pmc_current`)
  frame_roofline algorithmic TFLOP per frame (depth_completion_amd/flops.py, SURVEY §8d convention, at the
                 run's own latent shape, steps and seeds) x fps / 2.5 PF; `executed_*`: the same less the decoder
                 FLOPs the sparse-aware decode skips (its row-list launches against the dense decode)
  launches       kernel nodes of one captured guided step (hipGraphGetNodes)
  cpu_baseline   the oracle (CPU PyTorch restatement of the reference path, incl. weight-gradients as the
                 reference computes them) on this host's cores, rank 0 / N=1 only, on a bounded sample
                 (1- and 3-step calls, extrapolated to the run's steps / seeds)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md "Peak BF16/FP16 MFMA")
PEAK_CLOCK_HZ = 2.4e9    # the peak engine clock that figure assumes (2.5 PFLOP/s = 2.4 GHz x 1024 SIMDs x 1024 FLOP)
PEAK_HBM_GBS = 8000.0
METRIC = "dense-depth frames/sec at 768x576, 50 guided steps; 1 & 8 MI355X"


def log(msg: str) -> None:
    """progress on stderr (a long run keeps writing; the JSON line alone goes to stdout)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def synth_frame(h, w, n_points, seed, pattern="uniform"):
    """Seeded RGB (smooth gradient + noise) + 8-bit quantised sparse depth.
    pattern "beams": 64 scan rows evenly spaced over the lower 60 % of the image, each pixel kept with
    p = 0.25 (C4, KITTI-style 64-beam LiDAR); "uniform": n_points uniformly random pixels."""
    import torch
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, h), torch.linspace(0, 1, w), indexing="ij")
    img = (torch.stack([xx, yy, 0.5 * (xx + yy)]) * 200 + torch.randn((3, h, w), generator=g) * 12)
    img = img.clamp(0, 255).round().to(torch.uint8)
    field = 10 + 80 * yy + 20 * torch.sin(6.28 * xx + seed)
    k = (field * 255 / 120).round().clamp(1, 255)
    sp = torch.zeros(h * w)
    if pattern == "beams":
        rows = torch.linspace(0.4 * h, h - 1, 64).round().long()
        keep = torch.zeros(h, w, dtype=torch.bool)
        keep[rows] = torch.rand(64, w, generator=g) < 0.25
        idx = keep.view(-1).nonzero().view(-1)
    else:
        idx = torch.randperm(h * w, generator=g)[:n_points]
    sp[idx] = 120 * k.view(-1)[idx] / 255
    return img, sp.view(1, h, w)


def workload_name(h: int, w: int, batch: int, seeds: int) -> str:
    """BASELINE.json configs: C1 (384x384 @ res 768), C2 / C3 (768x576, 1 / 8 frames), C4 (KITTI 1216x352),
    C5 (nuScenes 1600x900, 10-seed ensemble); anything else is a custom shape."""
    if (h, w) == (576, 768) and seeds == 1:
        return "C2" if batch == 1 else "C3" if batch == 8 else f"C2-batch{batch}"
    if (h, w) == (384, 384):
        return "C1"
    if (h, w) == (352, 1216):
        return "C4"
    if (h, w) == (900, 1600):
        return "C5" if seeds == 10 else f"C5-shape ({seeds} seed(s))"
    return "custom"


def conv_flops(d, dense: bool = False) -> float:
    """Algorithmic FLOPs of one dc_conv_gemm launch (real channels, valid taps only; a row-list launch
    counts its rows, padding included; dense: as if it ran on the whole map)."""
    M = d.nrows if (d.rows and not dense) else d.nb * d.hout * d.wout
    K = d.kh * d.kw * d.cin
    f = 2.0 * M * d.cout * K
    if d.mode == 2:   # transposed stride-2 gather: on average 1/4 of the taps are valid
        f /= 4.0
    return f


def conv_bytes(d) -> float:
    """Algorithmic HBM bytes of one dc_conv_gemm launch: its input activations, weights, outputs and residual once
    each (bf16), what a launch must move if nothing were re-read (the floor the PMC traffic is compared with)."""
    M = d.nrows if d.rows else d.nb * d.hout * d.wout
    b = 2.0 * (d.nb * d.hin * d.win * d.cin + d.cout * d.kh * d.kw * d.cin + M * d.cout)
    if d.resid:
        b += 2.0 * M * d.cout
    return b


def measure_conv_kernel(pipe, st, reps: int = 3):
    """Time of the dominant kernel (dc_conv_gemm) inside one graph-replayed guided step.

    The step is captured twice as a hipGraph: as the timed region runs it, and with every
    dc_conv_gemm launch left out.  Each graph is replayed `reps` times between HIP events on the
    launch stream; the difference is the time the step spends in its conv launches, in the step's
    own order and cache state (no per-launch event packets).  Returns (launches, conv ms per step,
    algorithmic FLOPs per step, kernel nodes of the whole step, algorithmic bytes per step).
    """
    import torch
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

    nodes = {}

    def timed_graph(hook, count_nodes=False):
        g = torch.cuda.CUDAGraph(keep_graph=True) if count_nodes else torch.cuda.CUDAGraph()
        ops.call = hook
        try:
            with torch.cuda.graph(g):
                pipe._step(st)
        finally:
            ops.call = orig
        if count_nodes:
            g.instantiate()
            nodes.update(graph_node_counts(g.raw_cuda_graph()))
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
        t_all = timed_graph(record, count_nodes=True)
        n = len(descs)
        t_rest = timed_graph(skip_conv)
    finally:
        st["dec"].set_rows(None)
    flops = sum(conv_flops(d) for d in descs)
    # the FLOPs the sparse-aware decode's row-list launches skip against the dense decode SURVEY §8d counts
    skipped = sum(conv_flops(d, dense=True) - conv_flops(d) for d in descs if d.rows)
    return n, max(t_all - t_rest, 1e-6), flops, nodes, sum(conv_bytes(d) for d in descs), skipped


def graph_node_counts(raw_graph: int) -> dict:
    """Node counts by type of a captured hipGraph (kernel / memset / memcpy / other)."""
    import torch
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    n = ctypes.c_size_t(0)
    if hip.hipGraphGetNodes(ctypes.c_void_p(raw_graph), None, ctypes.byref(n)) != 0:
        return {}
    arr = (ctypes.c_void_p * n.value)()
    hip.hipGraphGetNodes(ctypes.c_void_p(raw_graph), arr, ctypes.byref(n))
    names = {0: "kernel", 1: "memcpy", 2: "memset"}
    out = {"total": int(n.value)}
    for node in arr:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(node), ctypes.byref(t))
        k = names.get(t.value, "other")
        out[k] = out.get(k, 0) + 1
    return out


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpu_quota():
    """The CPU quota of this process's cgroup as (label, CPUs): cgroup v2 cpu.max ("max 100000" = unlimited, or
    "<quota> <period>" microseconds), else cgroup v1 cfs_quota / cfs_period; CPUs None when unlimited or unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q == "max":
            return f"cpu.max {q} {per} (unlimited)", None
        return f"cpu.max {q} {per}", int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q <= 0:
            return f"cfs_quota_us {q} (unlimited)", None
        return f"cfs_quota_us {q} / cfs_period_us {per}", q / per
    except (OSError, ValueError):
        return "no cgroup CPU quota readable", None


def cpu_baseline(h, w, n_points, steps, seeds, pattern):
    """Oracle (CPU restatement) timed on this host: 1- and 3-step calls of one seed, extrapolated to the
    run's guided steps and seeds (an ensemble frame = `seeds` independent samples + a negligible fit)."""
    import torch
    from oracle import pipeline_ref as P
    from oracle.diffusers_ref import (AutoencoderTiny, DDIMScheduler, UNet2DConditionModel, synthetic_state_dict,
                                      synthetic_taesd_state_dict, synthetic_text_embedding)
    # the CPUs this process may run on (the reference's CPU path on the host's cores): the
    # affinity mask, capped by OMP_NUM_THREADS where the host declares its CPU share that way (the GPU boxes show
    # every CPU of the machine in the mask but give a job 16; more threads than that oversubscribe the share)
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = min(aff, int(omp)) if omp.isdigit() and int(omp) > 0 else aff
    quota_label, quota = cgroup_cpu_quota()
    if quota is not None:   # never more threads than the cgroup's CPU quota grants
        threads = max(1, min(threads, int(quota)))
    torch.set_num_threads(threads)
    # heartbeat on stderr while the oracle runs (a silent minute-long CPU leg must not look hung)
    import threading
    done = threading.Event()

    def beat():
        t0 = time.perf_counter()
        while not done.wait(30.0):
            log(f"cpu baseline: running ({time.perf_counter() - t0:.0f} s)")
    threading.Thread(target=beat, daemon=True).start()
    unet = UNet2DConditionModel()
    unet.load_state_dict(synthetic_state_dict(unet, 11))
    vae = AutoencoderTiny()
    vae.load_state_dict(synthetic_taesd_state_dict(vae, 12))
    pipe = P.OracleMarigoldDC(unet.to(torch.bfloat16), vae.to(torch.bfloat16), DDIMScheduler(),
                              synthetic_text_embedding(13, 1024), dtype=torch.bfloat16)
    img, sp = synth_frame(h, w, n_points, 0, pattern)
    # a 1-step call twice (the first also pays one-time allocation; the faster one counts), then a 3-step call: the
    # per-step time is half the 3-step / 1-step difference (a 1- / 2-step difference swung 0.6-2.1 s per step from
    # box to box)
    times = {}
    for s in (1, 1, 3):
        t0 = time.perf_counter()
        pipe(img[None], sp[None], 120.0, norm="const", steps=s, resolution=768)
        dt = time.perf_counter() - t0
        times[s] = min(times.get(s, dt), dt)
        log(f"cpu baseline: {s}-step oracle call {dt:.1f} s on {threads} threads")
    done.set()
    t_step = max((times[3] - times[1]) / 2.0, 1e-3)
    t_fixed = max(times[1] - t_step, 0.0)
    t_frame = (t_fixed + steps * t_step) * seeds
    return {"value": 1.0 / t_frame, "unit": "frames/s", "cores": threads,
            "cores_label": f"{threads} threads: affinity mask {aff} CPUs, OMP_NUM_THREADS {omp or 'unset'}, "
                           f"cgroup {quota_label}, {os.cpu_count()} host CPUs",
            "cgroup_cpu_quota": quota,
            "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"oracle bf16 CPU pipeline, 1 frame {w}x{h}, 1- and 3-step calls "
                      f"({times[1]:.1f}s, {times[3]:.1f}s) extrapolated to {steps} guided steps x {seeds} seed(s) "
                      f"({t_step:.2f} s/step incl. weight-grads)"}


def pmc_record(h, w, batch):
    """Committed PMC pass for this latent shape, or None: the pass over the graph-replayed step
    (profiles/pmc_step*.json, tools/pmc_step.py: the population measure_conv_kernel times) before the older
    eager-run passes (profiles/pmc_conv_gemm*.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_step*.json"))) + \
        sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_conv_gemm*.json")))
    for path in paths:
        with open(path) as f:
            rec = json.load(f)
        if rec.get("latent_shape") == [batch, h, w]:
            rec["_file"] = os.path.relpath(path, REPO)
            return rec
    return None


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed calls (bench steps)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="frames per call per GPU (C2: 1, C3: 8)")
    ap.add_argument("--height", type=int, default=576)
    ap.add_argument("--width", type=int, default=768)
    ap.add_argument("--points", type=int, default=500)
    ap.add_argument("--pattern", choices=("uniform", "beams"), default="uniform")
    ap.add_argument("--seeds", type=int, default=1, help="seed ensemble per frame (C5: 10)")
    ap.add_argument("--denoise-steps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--same-frame", action="store_true", help="replay one frame in every timed call")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / timing path only: gloo on CPU, a host matmul per frame instead of the pipeline")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv) -> int:
    """--gpus N without a launcher: start N rank processes (fresh interpreters; this parent never touches
    the GPU), wait for all, return the first non-zero exit status (the others are then terminated)."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in alive:
                    q.terminate()
        time.sleep(0.2)
    return rc


def run_worker(args) -> None:
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dry = args.dry_run
    if dry:
        dev = torch.device("cpu")
        torch.set_num_threads(1)
        if world > 1:
            dist.init_process_group("gloo")
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)

    from depth_completion_amd.flops import frame_flops
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    from depth_completion_amd.shard import frame_shard, max_over_ranks

    B, H, W, S = args.batch, args.height, args.width, args.seeds
    h, w = MarigoldDepthCompletionPipeline.latent_hw(H, W, 768)
    calls = args.warmup + args.steps
    # the job's frames: call c processes frames c*world*B .. (c+1)*world*B-1, contiguous shard per rank
    frame_sets = []
    for c in range(calls):
        base = 0 if args.same_frame else c * world * B
        fr = [synth_frame(H, W, args.points, seed=base + i, pattern=args.pattern)
              for i in frame_shard(world * B, rank, world)]
        frame_sets.append((torch.stack([f[0] for f in fr]).to(dev), torch.stack([f[1] for f in fr]).to(dev)))
    kw = dict(norm="const", steps=args.denoise_steps, resolution=768)

    if dry:
        wmat = torch.randn(256, 256)

        def run(imgs, sps):   # stands in for the pipeline: per-frame host work, no GPU
            x = imgs.float().flatten(1)[:, :256]
            for _ in range(200):
                x = torch.tanh(x @ wmat)
            return x, None
        pipe = None
    else:
        from depth_completion_amd import synthetic
        from depth_completion_amd.config import MARIGOLD_V1
        pipe = MarigoldDepthCompletionPipeline(synthetic.unet_state_dict(MARIGOLD_V1, 11),
                                               synthetic.taesd_state_dict(12), synthetic.text_embedding(13, 1024),
                                               device=dev, use_graph=not args.no_graph)
        if S > 1:
            seeds = list(range(2024, 2024 + S))

            def run(imgs, sps):
                d, _, lat = pipe.ensemble(imgs, sps, 120.0, seeds=seeds, **kw)
                return d, lat
        else:
            def run(imgs, sps):
                return pipe(imgs, sps, 120.0, **kw)

    def sync():
        if not dry:
            torch.cuda.synchronize(dev)

    log(f"rank {rank}/{world}: pipeline ready, {args.warmup} warm-up + {args.steps} timed calls")
    for c in range(args.warmup):
        run(*frame_sets[c])
    sync()
    log(f"rank {rank}: warm-up done")
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for c in range(args.warmup, calls):
        dense, _ = run(*frame_sets[c])
    sync()
    log(f"rank {rank}: timed calls done ({time.perf_counter() - t0:.2f} s)")
    if world > 1:
        dist.barrier()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine, device=None if dry else dev)
    # who ran: every rank's (rank, LOCAL_RANK, device PCI address, elapsed) -- the 8-GPU line then shows 8
    # distinct ranks on 8 distinct devices
    if dry:
        devname = "cpu"
    else:
        pr = torch.cuda.get_device_properties(dev)
        devname = (f"{getattr(pr, 'pci_domain_id', 0):04x}:{getattr(pr, 'pci_bus_id', 0):02x}:"
                   f"{getattr(pr, 'pci_device_id', 0):02x}")
    me = {"rank": rank, "local_rank": local, "device": devname, "elapsed_s": mine}
    ranks = [me]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    per_rank = [r["elapsed_s"] for r in ranks]
    rccl_world = dist.get_world_size() if (world > 1 and dist.is_initialized()) else 1
    assert torch.isfinite(dense).all(), "non-finite dense output"

    frames_total = world * args.steps * B
    value = frames_total / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    ff = frame_flops(h, w, args.denoise_steps, S)
    frame_tflop = ff["per_frame"] / 1e12
    fps_gpu = value / world
    line = {
        "metric": METRIC, "value": round(value, 4), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2), "ms_per_frame": round(1000.0 / fps_gpu, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (seeded RGB + 8-bit quantised sparse depth; seeded synthetic weights)",
        "config": {"workload": f"{workload_name(H, W, B, S)}: {W}x{H} RGB + "
                               f"{'64-beam' if args.pattern == 'beams' else str(args.points) + '-pt'} sparse depth, "
                               f"{args.denoise_steps} guided DDIM steps, {B} frame(s) per call per GPU"
                               + (f", {S}-seed ensemble + affine fit per frame" if S > 1 else ""),
                   "frames_per_step": B * world, "seeds_per_frame": S, "resolution": 768, "latent": [h, w],
                   "guided_steps": args.denoise_steps, "parallelism": f"frame-sharded dp{world} (no collectives)",
                   "weights": "synthetic seeded (Marigold v1-0 UNet + TAESD shapes)",
                   "hip_graph": not args.no_graph, "distinct_frames_per_call": not args.same_frame},
        "per_rank_fps": [round(args.steps * B / t, 4) for t in per_rank],
        "rccl_world": rccl_world,
        "ranks": [{"rank": r["rank"], "local_rank": r["local_rank"], "device": r["device"],
                   "fps": round(args.steps * B / r["elapsed_s"], 4)} for r in ranks],
        "max_over_ranks_s": round(elapsed, 6),
        "frame_roofline": {"algorithmic_tflop_per_frame": round(frame_tflop, 2),
                           "achieved_tflops_per_gpu": round(fps_gpu * frame_tflop, 2),
                           "frac_of_bf16_peak": round(fps_gpu * frame_tflop / PEAK_BF16_TFLOPS, 4),
                           "ceiling_fps_per_gpu": round(PEAK_BF16_TFLOPS / frame_tflop, 3),
                           "convention": "SURVEY §8d (fwd + input-grad, attention bwd = 2x fwd), "
                                         "depth_completion_amd/flops.py at this latent shape"},
    }
    if dry:
        line["dry_run"] = True
        line["dtype"] = "f32"
        del line["frame_roofline"]
    elif rank == 0:
        st = pipe._plans[(B * S, h, w)]
        n_launch, conv_ms, conv_flops_, nodes, conv_bytes_, skipped = measure_conv_kernel(pipe, st)
        # the frame's executed work: SURVEY's count less what the sparse-aware decode never computes (its row-list
        # launches cover the resize taps' receptive fields only), so the sparse decode does not inflate the fraction
        exec_tflop = (ff["per_frame"] - skipped * args.denoise_steps / B) / 1e12
        line["frame_roofline"].update(executed_tflop_per_frame=round(exec_tflop, 2),
                                      executed_frac_of_bf16_peak=round(fps_gpu * exec_tflop / PEAK_BF16_TFLOPS, 4))
        avg_ms = conv_ms / max(n_launch, 1)
        achieved = conv_flops_ / (conv_ms * 1e-3) / 1e12
        roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": None,
                    "kernel": "dc_conv_gemm = conv_gemm_kernel, implicit-GEMM conv/linear (all instantiations)",
                    "launches_per_step": n_launch, "avg_launch_ms": round(avg_ms, 5),
                    "method": "graph-replayed step minus the same graph without its conv launches (HIP events)",
                    "algorithmic_gflop_per_step": round(conv_flops_ / 1e9, 1),
                    "algorithmic_bytes_per_step": round(conv_bytes_)}
        pmc = pmc_record(h, w, B * S)
        if pmc is not None:
            t = pmc["traffic_bytes_per_launch"]
            roofline.update(traffic=round(t), traffic_unit="HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)",
                            hbm_gbs=round(t / (avg_ms * 1e-3) / 1e9, 1), pmc_source=pmc["_file"])
            if pmc.get("traffic_bytes_per_step") is not None:
                roofline["traffic_per_step"] = round(pmc["traffic_bytes_per_step"])
                # counter bytes over the launches' own operands moved once: the re-fetch factor beyond L2
                roofline["traffic_over_algorithmic"] = round(pmc["traffic_bytes_per_step"] / conv_bytes_, 2)
            from depth_completion_amd.build import conv_family_hash
            current = pmc.get("conv_family_hash") == conv_family_hash()
            roofline["pmc_current"] = current   # counters taken on this tree's conv kernels and tuned table
            if pmc.get("mfma_busy_cycles_per_step") is not None and current:
                # MFMA-busy cycles of the step's conv family over that family's graph-replayed time at the peak
                # clock x 1024 SIMDs: one v_mfma_f32_16x16x32_bf16 (16 K FLOP) keeps a SIMD busy 16 cycles, so this
                # is >= frac by construction (it counts padding and split-hi/lo MFMAs that frac does not)
                roofline["mfma_util"] = round(pmc["mfma_busy_cycles_per_step"] /
                                              (conv_ms * 1e-3 * PEAK_CLOCK_HZ * 1024), 4)
                roofline["mfma_util_def"] = ("PMC SQ_VALU_MFMA_BUSY_CYCLES per step / (graph-timed family ms x "
                                             "2.4 GHz x 1024 SIMDs)")
            if pmc.get("mfma_util_pmc_window") is not None:
                roofline["mfma_util_pmc_window"] = round(pmc["mfma_util_pmc_window"], 4)
        line["roofline"] = roofline
        line["launches"] = {"kernel_nodes_per_guided_step": nodes.get("kernel"), "graph_nodes": nodes}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not dry:
        log("cpu baseline (oracle on the host cores)")
        line["cpu_baseline"] = cpu_baseline(H, W, args.points, args.denoise_steps, S, args.pattern)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ and args.gpus != 1:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    run_worker(args)


if __name__ == "__main__":
    main()

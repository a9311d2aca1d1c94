"""Measure the fastest dc_conv_gemm variant for every conv/linear shape of the sampler (GPU).

The committed table is tuned with DC_TUNE_COLD=1 (caches flushed before every timed call).

Runs one eager guided call per workload with Ctx.tune on (each new shape is timed over all tile
algos x split-K on its real operands) and writes the table that ops.load_tuned() reads.

Usage: python tools/tune_gemm.py [--workloads c2:1 c2:8 c4:1 c4:8 c5:1] [--out depth_completion_amd/tuned_gfx950.json]
       [--try 37 38 ...]  (the committed choices against new variants only)
  workload:batch -- c2 / c3: 768x576, 500 uniform points; c4: 1216x352, 64-beam rows; c5: 1600x900, 3000
  points, run as the 10-seed ensemble (one batch-10 call per frame, the shapes C5 launches)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_frame  # noqa: E402
from depth_completion_amd import ops, synthetic  # noqa: E402
from depth_completion_amd.config import MARIGOLD_V1  # noqa: E402
from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", nargs="+", default=["c2:1", "c2:8"])
    ap.add_argument("--out", default="gpurun_out/tuned_gfx950.json")
    ap.add_argument("--fresh", action="store_true", help="ignore the committed table")
    ap.add_argument("--retune-3x3", action="store_true",
                    help="re-time the stride-1 3x3 shapes with cin %% 64 == 0 (the halo-kernel contract) over every "
                         "variant, keep the committed choice of every other shape")
    ap.add_argument("--try", dest="try_algos", type=int, nargs="+",
                    help="re-time every shape of the workloads: its committed choice against these algo ids (all "
                         "their splits) only; shapes outside the workloads keep their entries")
    ap.add_argument("--top-out", help="also write every re-timed shape's six fastest variants (isolated timing) here, "
                    "the candidates tools/ab/instep_tables.py evaluates inside the step")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    pipe = MarigoldDepthCompletionPipeline(synthetic.unet_state_dict(MARIGOLD_V1, 11), synthetic.taesd_state_dict(12),
                                           synthetic.text_embedding(13, 1024), device=dev, use_graph=False)
    if args.fresh:
        pipe.ctx.algo_cache = {}
    if args.retune_3x3:
        # key = (mode, nb, hin, win, cin, hout, wout, cout, kh, stride, two_src, ktot) (ops.conv_key)
        keep = {k: v for k, v in pipe.ctx.algo_cache.items()
                if not (k[8] == 3 and k[9] == 1 and k[4] % 64 == 0 and k[0] in (0, 1))}
        print(f"re-tuning {len(pipe.ctx.algo_cache) - len(keep)} 3x3 shapes", flush=True)
        pipe.ctx.algo_cache = keep
    committed = dict(pipe.ctx.algo_cache)
    if args.try_algos:
        pipe.ctx.tune_only = (set(args.try_algos), committed)
        pipe.ctx.algo_cache = {}
    pipe.ctx.tune = True
    if args.top_out:
        pipe.ctx.tune_top = {}
    shapes = {"c2": (576, 768, 500, "uniform"), "c3": (576, 768, 500, "uniform"), "c4": (352, 1216, 0, "beams"),
              "c5": (900, 1600, 3000, "uniform")}
    for wl in args.workloads:
        name, b = wl.split(":")
        h, w, npts, pattern = shapes[name]
        fr = [synth_frame(h, w, npts, i, pattern) for i in range(int(b))]
        imgs = torch.stack([f[0] for f in fr]).to(dev)
        sps = torch.stack([f[1] for f in fr]).to(dev)
        n0 = len(pipe.ctx.algo_cache)
        if name == "c5":
            pipe.ensemble(imgs, sps, 120.0, seeds=list(range(2024, 2034)), norm="const", steps=2, resolution=768)
        else:
            pipe(imgs, sps, 120.0, norm="const", steps=2, resolution=768)
        torch.cuda.synchronize()
        print(f"{wl}: {len(pipe.ctx.algo_cache) - n0} new shapes tuned", flush=True)
        ops.save_tuned(pipe.ctx.algo_cache, args.out)   # keep what is done if a later workload is cut off
    if args.try_algos:
        changed = sum(1 for k, v in pipe.ctx.algo_cache.items() if committed.get(k) != v)
        print(f"--try {args.try_algos}: {changed} of {len(pipe.ctx.algo_cache)} re-timed shapes changed", flush=True)
        pipe.ctx.algo_cache = {**committed, **pipe.ctx.algo_cache}
    ops.save_tuned(pipe.ctx.algo_cache, args.out)
    if args.top_out:
        with open(args.top_out, "w") as f:
            json.dump([{"key": list(k), "top": [list(c) for c in v]} for k, v in sorted(pipe.ctx.tune_top.items())], f)
    for k, v in sorted(pipe.ctx.algo_cache.items()):
        print(k, v)


if __name__ == "__main__":
    main()

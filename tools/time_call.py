"""Break one C2 guided call into phases: host time vs device time (GPU).

Times (a) a full call, (b) 50 bare graph replays of the captured step, (c) one eager step, and
(d) host-side time of g.replay() itself, to separate per-call overhead, the step's kernels and
launch gaps.

Usage: python tools/time_call.py [--batch 1]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_frame  # noqa: E402
from depth_completion_amd import synthetic  # noqa: E402
from depth_completion_amd.config import MARIGOLD_V1  # noqa: E402
from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    pipe = MarigoldDepthCompletionPipeline(synthetic.unet_state_dict(MARIGOLD_V1, 11), synthetic.taesd_state_dict(12),
                                           synthetic.text_embedding(13, 1024), device=dev)
    fr = [synth_frame(576, 768, 500, i) for i in range(args.batch)]
    imgs = torch.stack([f[0] for f in fr]).to(dev)
    sps = torch.stack([f[1] for f in fr]).to(dev)
    kw = dict(norm="const", steps=50, resolution=768)
    pipe(imgs, sps, 120.0, **kw)
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    pipe(imgs, sps, 120.0, **kw)
    torch.cuda.synchronize()
    t_call = time.perf_counter() - t0

    st = pipe._plans[(args.batch, pipe._call_state["h"], pipe._call_state["w"])]
    g = st["graph"]
    pipe.ctx.step.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        g.replay()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_graph = time.perf_counter() - t0

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pipe.ctx.step.zero_()
    e0.record()
    pipe._step(st)
    e1.record()
    torch.cuda.synchronize()
    t_eager = e0.elapsed_time(e1)

    # one replay alone (best of 5) against a back-to-back chain of 50, both between HIP events
    one = []
    for _ in range(5):
        pipe.ctx.step.zero_()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        one.append(e0.elapsed_time(e1))
    pipe.ctx.step.zero_()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(50):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    chain = e0.elapsed_time(e1) / 50

    print(f"full call {t_call*1e3:.1f} ms | 50 graph replays {t_graph*1e3:.1f} ms (host enqueue {t_host*1e3:.1f} ms)"
          f" -> {t_graph / 50 * 1e3:.2f} ms/step | eager step {t_eager:.2f} ms | per-call overhead "
          f"~{(t_call - t_graph) * 1e3:.1f} ms | one replay {min(one):.3f} ms (events, best of 5), chained "
          f"{chain:.3f} ms/replay", flush=True)


if __name__ == "__main__":
    main()

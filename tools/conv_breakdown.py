"""Per-launch breakdown of dc_conv_gemm over one guided C2 step (GPU).

Each conv launch of the step is replayed 10x inside a small hipGraph between HIP events (as in
bench.py's roofline leg); prints shapes grouped by (M, N, K, mode) with total time and TF/s.
Usage: python tools/conv_breakdown.py [--batch 1] [--tune]
"""
import argparse
import ctypes as C
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import conv_flops, synth_frame  # noqa: E402
from depth_completion_amd import _lib, ops, synthetic  # noqa: E402
from depth_completion_amd._lib import ConvDesc  # noqa: E402
from depth_completion_amd.config import MARIGOLD_V1  # noqa: E402
from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    pipe = MarigoldDepthCompletionPipeline(synthetic.unet_state_dict(MARIGOLD_V1, 11), synthetic.taesd_state_dict(12),
                                           synthetic.text_embedding(13, 1024), device=dev, use_graph=False)
    fr = [synth_frame(576, 768, 500, i) for i in range(args.batch)]
    imgs = torch.stack([f[0] for f in fr]).to(dev)
    sps = torch.stack([f[1] for f in fr]).to(dev)
    pipe(imgs, sps, 120.0, norm="const", steps=1, resolution=768)
    st = pipe._plans[(args.batch, pipe._call_state["h"], pipe._call_state["w"])]
    descs = []
    orig = ops.call

    def rec(name, *a):
        if name == "dc_conv_gemm":
            descs.append(ConvDesc.from_buffer_copy(a[0]._obj))
        return orig(name, *a)

    ops.call = rec
    ops.memset(pipe.ctx, pipe.ctx.step)
    pipe._step(st)
    ops.call = orig
    torch.cuda.synchronize()
    groups = defaultdict(lambda: [0, 0.0, 0.0, None])
    tot_ms = 0.0
    for d in descs:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                _lib.call("dc_conv_gemm", C.byref(d), torch.cuda.current_stream().cuda_stream)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 10
        M = d.nb * d.hout * d.wout
        key = (M, d.cout, d.kh * d.kw * d.cin, d.mode, d.kh)
        gr = groups[key]
        gr[0] += 1
        gr[1] += ms
        gr[2] += conv_flops(d)
        gr[3] = ops.Ctx.choose_algo(pipe.ctx, d)
        tot_ms += ms
    print(f"{len(descs)} launches, {tot_ms:.3f} ms per step")
    for key, (n, ms, fl, alg) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        M, N, K, mode, k = key
        print(f"M={M:7d} N={N:5d} K={K:6d} mode={mode} k={k} x{n:3d}: {ms*1e3:8.1f} us total "
              f"({100*ms/tot_ms:5.1f} %), {fl/ms/1e9:6.1f} TF/s, algo {alg}", flush=True)


if __name__ == "__main__":
    main()

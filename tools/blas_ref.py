"""Headroom check: dc_conv_gemm vs torch.matmul (hipBLASLt) on the sampler's GEMM shapes (GPU).

For each shape of tools/bench_gemm.py the plain GEMM equivalent (M = output pixels, N = cout,
K = taps x cin) is timed with torch.matmul in bf16, and dc_conv_gemm on the real conv (implicit
im2col) with its tuned / autotuned variant.  Both are captured 20x in a hipGraph and replayed between
HIP events; "cold" flushes L2 + the Infinity Cache (512 MiB write) before a single timed call.
Usage: python tools/blas_ref.py
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import SHAPES  # noqa: E402

dev = torch.device("cuda:0")


def graph_time(fn, reps=20):
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def cold_time(fn, flush, reps=5):
    t = 0.0
    for _ in range(reps):
        flush.fill_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        t += e0.elapsed_time(e1)
    return t / reps


def main():
    ctx = Ctx(dev, tune=True)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    print(f"{'shape':18s} {'M':>7s} {'N':>6s} {'K':>6s} | {'blas warm':>9s} {'ours warm':>9s} | "
          f"{'blas cold':>9s} {'ours cold':>9s}   (TF/s)", flush=True)
    for name, nb, h, w, cin, cout, k, stride, mode in SHAPES:
        hin, win = (h // 2, w // 2) if mode == 1 else (h, w)
        ho, wo = ((h + 2 - 3) // stride + 1, (w + 2 - 3) // stride + 1) if k == 3 else (h, w)
        M, N, K = nb * ho * wo, cout, k * k * cin
        flops = 2.0 * M * N * K
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        bt = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def blas():
            torch.matmul(a, bt.t(), out=c)
        x = torch.randn(nb * hin * win, cin, device=dev).to(torch.bfloat16)
        ktot = -(-K // 64) * 64
        wt = (torch.randn(cout, ktot, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        bias = torch.zeros(cout, device=dev)

        def ours():
            ops.conv_gemm(ctx, x, wt, nb=nb, hin=hin, win=win, cin=cin, hout=ho, wout=wo, cout=cout, kh=k, kw=k,
                          stride=stride, pad=1 if k == 3 else 0, mode=mode, bias=bias, y=y)
        ours()   # autotunes the shape if the committed table lacks it
        tb, to = graph_time(blas), graph_time(ours)
        cb, co = cold_time(blas, flush), cold_time(ours, flush)
        print(f"{name:18s} {M:7d} {N:6d} {K:6d} | {flops / tb / 1e9:9.1f} {flops / to / 1e9:9.1f} | "
              f"{flops / cb / 1e9:9.1f} {flops / co / 1e9:9.1f}   us: {tb*1e3:.1f} {to*1e3:.1f} {cb*1e3:.1f} "
              f"{co*1e3:.1f}", flush=True)


if __name__ == "__main__":
    main()

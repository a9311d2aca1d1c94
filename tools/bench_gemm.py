"""Microbenchmark of dc_conv_gemm on the UNet's representative shapes (GPU).

Usage: python tools/bench_gemm.py [--reps N]
Prints TFLOP/s per shape (algorithmic FLOPs / avg kernel time from HIP events).
"""
import argparse
import math
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

dev = torch.device("cuda:0")
from depth_completion_amd import _lib  # noqa: E402
NALG = _lib.load().dc_conv_num_algos()

# (name, nb, h, w, cin, cout, k, stride, mode)
SHAPES = [
    ("big4096_linear", 1, 1, 4096, 4096, 4096, 1, 1, 0),
    ("L0_proj320", 1, 1, 6912, 320, 320, 1, 1, 0),
    ("L2_proj1280", 1, 1, 432, 1280, 1280, 1, 1, 0),
    ("L0_conv320", 1, 72, 96, 320, 320, 3, 1, 0),
    ("L0_conv640in", 1, 72, 96, 640, 320, 3, 1, 0),
    ("L1_conv640", 1, 36, 48, 640, 640, 3, 1, 0),
    ("L2_conv1280", 1, 18, 24, 1280, 1280, 3, 1, 0),
    ("L3_conv1280", 1, 9, 12, 1280, 1280, 3, 1, 0),
    ("L3_conv2560in", 1, 9, 12, 2560, 1280, 3, 1, 0),
    ("L0_ff1", 1, 1, 6912, 320, 2560, 1, 1, 0),
    ("L0_ff2", 1, 1, 6912, 1280, 320, 1, 1, 0),
    ("L0_qkv", 1, 1, 6912, 320, 960, 1, 1, 0),
    ("L1_ff1", 1, 1, 1728, 640, 5120, 1, 1, 0),
    ("L2_ff1", 1, 1, 432, 1280, 10240, 1, 1, 0),
    ("L0_up_conv640", 1, 72, 96, 640, 640, 3, 1, 1),
    ("taesd_full64", 1, 576, 768, 64, 64, 3, 1, 0),
    ("taesd_288_64", 1, 288, 384, 64, 64, 3, 1, 0),
    ("L0_conv320_b8", 8, 72, 96, 320, 320, 3, 1, 0),
    ("L2_conv1280_b8", 8, 18, 24, 1280, 1280, 3, 1, 0),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    ctx = Ctx(dev)
    tot_t = 0.0
    for name, nb, h, w, cin, cout, k, stride, mode in SHAPES:
        hin, win = (h // 2, w // 2) if mode == 1 else (h, w)
        x = torch.randn(nb * hin * win, cin, device=dev).to(torch.bfloat16)
        ktot = -(-(k * k * cin) // 64) * 64
        wt = (torch.randn(cout, ktot, device=dev) / math.sqrt(k * k * cin)).to(torch.bfloat16)
        ho, wo = ((h + 2 - 3) // stride + 1, (w + 2 - 3) // stride + 1) if k == 3 else (h, w)
        y = torch.empty(nb * ho * wo, cout, device=dev, dtype=torch.bfloat16)
        b = torch.zeros(cout, device=dev)

        flops = 2.0 * nb * ho * wo * cout * k * k * cin
        res = []
        for algo, ns in [(0, 0)] + [(a, s) for a in range(1, NALG + 1) for s in (1, 2, 4, 8, 16, -1, -2, -3)]:
            def run():
                ops.conv_gemm(ctx, x, wt, nb=nb, hin=hin, win=win, cin=cin, hout=ho, wout=wo, cout=cout, kh=k,
                              kw=k, stride=stride, pad=k // 2, mode=mode, bias=b, y=y, algo=algo, nsplit=ns)

            for _ in range(2):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            res.append((ms, algo, ns))
        auto_ms = res[0][0]
        best = min(r for r in res if r[2] >= 0)
        bsk = min(r for r in res if r[2] < 0)
        print(f"{name:18s} M={nb*ho*wo:7d} N={cout:6d} K={k*k*cin:6d}  auto {auto_ms*1e3:8.1f} us "
              f"{flops/auto_ms/1e9:7.1f} TF | best split-K algo {best[1]} split {best[2]} {best[0]*1e3:8.1f} us "
              f"{flops/best[0]/1e9:7.1f} TF | best stream-K algo {bsk[1]} G {-bsk[2] * 256} {bsk[0]*1e3:8.1f} us "
              f"{flops/bsk[0]/1e9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()

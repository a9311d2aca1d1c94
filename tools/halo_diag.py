"""Halo-kernel diagnostics: time one conv shape with parts of the kernel switched off (DC_HALO_DIAG bits:
1 no LDS-DMA issue, 2 no fragment reads / MFMAs, 4 no barrier) to see what bounds an iteration (GPU)."""
import ctypes as C
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import _lib, ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402


def timed(d, reps=20):
    g = torch.cuda.CUDAGraph()
    _lib.call("dc_conv_gemm", C.byref(d), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(reps):
            _lib.call("dc_conv_gemm", C.byref(d), torch.cuda.current_stream().cuda_stream)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


dev = torch.device("cuda:0")
ctx = Ctx(dev)
for (nb, h, w, cin, cout) in ((1, 72, 96, 64, 256), (1, 72, 96, 320, 256), (1, 72, 96, 640, 256),
                              (1, 72, 96, 1280, 256)):
    x = torch.randn(nb * h * w, cin, device=dev).to(torch.bfloat16)
    wt = (torch.randn(cout, 9 * cin, device=dev) / math.sqrt(9 * cin)).to(torch.bfloat16)
    y = torch.empty(nb * h * w, cout, device=dev, dtype=torch.bfloat16)
    for algo in (32, 24):
        res = []
        diags = (0, 1, 2, 3, 7, 15, 16, 32, 11)
        for diag in diags:
            os.environ["DC_HALO_DIAG"] = str(diag)
            d = ops.conv_desc(ctx, x, wt, nb=nb, hin=h, win=w, cin=cin, hout=h, wout=w, cout=cout, y=y, algo=algo,
                              nsplit=1)
            res.append(timed(d))
        print(f"{h}x{w} cin={cin} cout={cout} algo {algo}: " + " ".join(f"d{k}={t:6.1f}" for k, t in zip(diags, res)),
              flush=True)
    os.environ["DC_HALO_DIAG"] = "0"

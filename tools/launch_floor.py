"""Per-launch floor of dc_conv_gemm inside a hipGraph (GPU): 40 back-to-back launches of the M = 6912, N = 320 linear
as an empty kernel (DC_HALO_DIAG=128: return at entry), at K = 64 (one k-chunk), K = 64 without epilogue stores, and
K = 320, next to a chain of tiny torch kernels.  Run it under different HIP_* environment settings to compare
(e.g. HIP_FORCE_DEV_KERNARG)."""
import ctypes as C
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import _lib, ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402


def graph_us(fn, n=40):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return best


def main():
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    M, N = 6912, 320
    res = {}
    small = torch.zeros(1024, device=dev)
    res["torch add_ (4 blocks)"] = graph_us(lambda: small.add_(1.0))
    sb = torch.zeros(4096, dtype=torch.bfloat16, device=dev)
    res["dc_silu 4096 (libdcamd)"] = graph_us(
        lambda: _lib.call("dc_silu", sb.data_ptr(), sb.numel(), sb.data_ptr(), torch.cuda.current_stream().cuda_stream))
    for K in (64, 320):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for algo in (13, 12):
            for diag in ((128, 64, 0) if K == 64 else (0,)):
                os.environ["DC_HALO_DIAG"] = str(diag)
                d = ops.conv_desc(ctx, x, w, nb=1, hin=1, win=M, cin=K, hout=1, wout=M, cout=N, kh=1, kw=1, pad=0,
                                  y=y, algo=algo, nsplit=1)
                os.environ["DC_HALO_DIAG"] = "0"
                res[f"K={K} algo {algo} diag {diag}"] = graph_us(
                    lambda: _lib.call("dc_conv_gemm", C.byref(d), torch.cuda.current_stream().cuda_stream))
    env = {k: v for k, v in os.environ.items() if k.startswith("HIP_") or k.startswith("GPU_")}
    print("env", env)
    for k, v in res.items():
        print(f"{k:32s} {v:7.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()

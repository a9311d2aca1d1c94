"""Where the time of a short-K linear goes (GPU): one (M, K, N) linear timed as 20 launches in one hipGraph,
each launch on a different weight copy (weights cold, activations warm, as in the step), for a set of
variants, with and without the epilogue stores (DC_HALO_DIAG=64), and at K = 64 (one k-chunk: the launch floor).
Usage: python tools/lin_diag.py [--shapes M,K,N ...] [--algos a:s ...]"""
import argparse
import ctypes as C
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import _lib, ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402


def timed(descs):
    s = torch.cuda.current_stream().cuda_stream
    for d in descs[:2]:
        _lib.call("dc_conv_gemm", C.byref(d), s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for d in descs:
            _lib.call("dc_conv_gemm", C.byref(d), torch.cuda.current_stream().cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / len(descs) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["6912,320,320", "1728,640,640", "432,1280,1280",
                                                    "6912,320,960", "6912,320,2560", "6912,1280,320"])
    ap.add_argument("--algos", nargs="+", default=["13:1", "42:1", "37:1", "12:1", "38:1", "3:1", "18:1",
                                                   "59:1", "60:1", "61:1", "40:1", "39:1"])
    ap.add_argument("--copies", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    for sh in a.shapes:
        M, K, N = map(int, sh.split(","))
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ws = [(torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16) for _ in range(a.copies)]
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        b = torch.zeros(N, device=dev)
        x1 = x[:, :64].contiguous()
        ws1 = [w[:, :64].contiguous() for w in ws]
        line = []
        for al in a.algos:
            algo, sp = map(int, al.split(":"))
            res = []
            for diag, xx, wl in ((0, x, ws), (64, x, ws), (0, x1, ws1)):
                os.environ["DC_HALO_DIAG"] = str(diag)
                kk = xx.shape[1]
                descs = [ops.conv_desc(ctx, xx, w, nb=1, hin=1, win=M, cin=kk, hout=1, wout=M, cout=N, kh=1, kw=1,
                                       pad=0, bias=b, y=y, algo=algo, nsplit=sp) for w in wl]
                try:
                    res.append(timed(descs))
                except Exception as e:  # noqa: BLE001
                    res.append(float("nan"))
                    print("error", algo, sp, e, flush=True)
            os.environ["DC_HALO_DIAG"] = "0"
            tf = 2.0 * M * N * K / (res[0] * 1e-6) / 1e12
            line.append(f"  ({algo:2d},{sp:2d}) {res[0]:6.2f} us ({tf:5.0f} TF/s)  no-epi {res[1]:6.2f}  K=64 {res[2]:6.2f}")
        print(f"M={M} K={K} N={N}", flush=True)
        print("\n".join(line), flush=True)


if __name__ == "__main__":
    main()

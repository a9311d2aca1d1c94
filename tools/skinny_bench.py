"""Time the weight-streaming skinny conv / linear variants against the tuned choice on the batch-1 level-2 / 3 shapes.

Every launch in the timed graph reads its own copy of the weights (copies rotate over > 2x the 256 MB Infinity
Cache), so the weights stream from HBM as they do in the sampler step, where each layer's weights are touched once
per pass.  For each shape: the committed table's (algo, split), then every skinny algo x split; the output's
relative error against the tuned launch is a quick correctness screen (tests/test_gpu_kernels.py has the real tests).
Reports us per launch, TF/s and the weight-stream rate (weight bytes / time).
Usage: python tools/skinny_bench.py [--reps 20] [--set l2|l3|taesd|all] [--algos 43 44 ...] [--copies N] [--tuned-only]
(--copies N: rotate N weight copies instead -- 1 or 2 leave the weights in the Infinity Cache: warm against cold)
(taesd: the 64-channel decoder convs, for the weight-resident persistent variants, algo ids 55..)
"""
import argparse
import ctypes as C
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import _lib, ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

SKINNY_FIRST = 43   # dc_conv_gemm algo id of the first skinny variant (ops.SKINNY_FIRST)

# 3x3: (nb, hin, win, cin, hout, wout, cout, mode); linear: ("lin", rows, k, n)
L2 = [(1, 18, 24, 1280, 18, 24, 1280, 0), (1, 18, 24, 2560, 18, 24, 1280, 0), (1, 18, 24, 1280, 18, 24, 2560, 0),
      (1, 9, 12, 1280, 18, 24, 1280, 1), (1, 18, 24, 640, 18, 24, 1280, 0), (1, 18, 24, 1280, 18, 24, 640, 0),
      ("lin", 432, 1280, 1280), ("lin", 432, 10240, 1280), ("lin", 432, 5120, 1280), ("lin", 432, 1280, 3840),
      ("lin", 432, 3840, 1280), ("lin", 432, 2560, 1280)]
TAESD = [(1, 288, 384, 64, 288, 384, 64, 0), (1, 144, 192, 64, 288, 384, 64, 1), (1, 144, 192, 64, 144, 192, 64, 0),
         (1, 72, 96, 64, 144, 192, 64, 1), (1, 72, 96, 64, 72, 96, 64, 0)]
L3 = [(1, 9, 12, 1280, 9, 12, 1280, 0), (1, 9, 12, 2560, 9, 12, 1280, 0), (1, 9, 12, 1280, 9, 12, 2560, 0),
      ("lin", 108, 1280, 1280), ("lin", 108, 2560, 1280), ("lin", 108, 1280, 2560), ("lin", 108, 10240, 1280),
      ("lin", 108, 5120, 1280), ("lin", 108, 3840, 1280)]


def timed(descs, reps):
    """us per launch of a graph that cycles through ``descs`` (one weight copy each)."""
    st = torch.cuda.current_stream().cuda_stream
    for d in descs[:2]:
        _lib.call("dc_conv_gemm", C.byref(d), st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(reps):
                _lib.call("dc_conv_gemm", C.byref(descs[i % len(descs)]), s.cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--set", default="all")
    ap.add_argument("--algos", type=int, nargs="*")
    ap.add_argument("--copies", type=int, default=0)
    ap.add_argument("--tuned-only", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    nalg = _lib.load().dc_conv_num_algos()
    algos = args.algos or list(range(SKINNY_FIRST, nalg + 1))
    shapes = {"l2": L2, "l3": L3, "taesd": TAESD, "all": L2 + L3}[args.set]
    torch.manual_seed(0)
    for sh in shapes:
        if sh[0] == "lin":
            _, rows, k, n = sh
            nb, hin, win, cin, hout, wout, cout, mode, kk, pad = 1, 1, rows, k, 1, rows, n, 0, 1, 0
        else:
            nb, hin, win, cin, hout, wout, cout, mode = sh
            kk, pad = 3, 1
        ktot = kk * kk * cin
        wbytes = cout * ktot * 2
        ncopy = args.copies or max(2, min(args.reps, math.ceil(600e6 / wbytes)))
        x = torch.randn(nb * hin * win, cin, device=dev).to(torch.bfloat16)
        ws = [(torch.randn(cout, ktot, device=dev) / math.sqrt(ktot)).to(torch.bfloat16) for _ in range(ncopy)]
        b = torch.randn(cout, device=dev)
        y = torch.zeros(nb * hout * wout, cout, device=dev, dtype=torch.bfloat16)
        kw = dict(nb=nb, hin=hin, win=win, cin=cin, hout=hout, wout=wout, cout=cout, kh=kk, kw=kk, pad=pad, mode=mode,
                  bias=b, y=y)
        d0 = ops.conv_desc(ctx, x, ws[0], **kw)
        tuned = (d0.algo, d0.splitk)

        def descs(a, s):
            out = []
            for w in ws:
                d = ops.conv_desc(ctx, x, w, algo=a, nsplit=s, **kw)
                out.append(d)
            return out
        t0 = timed(descs(*tuned), args.reps)
        y.zero_()
        _lib.call("dc_conv_gemm", C.byref(descs(*tuned)[0]), torch.cuda.current_stream().cuda_stream)
        ref = y.float().clone()
        flops = 2.0 * nb * hout * wout * cout * ktot
        name = f"{'lin' if kk == 1 else 'c3'} M={nb * hout * wout} N={cout} K={ktot}" + (" up" if mode == 1 else "")
        print(f"{name:32s} tuned {tuned}: {t0:7.1f} us  {flops / t0 / 1e6:6.1f} TF/s  {wbytes / t0 / 1e3:7.1f} GB/s",
              flush=True)
        best = (t0, tuned)
        for a in ([] if args.tuned_only else algos):
            for s in (1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, -4, -6, -8, -10, -12, -16, -20):
                try:
                    ds = descs(a, s)
                    y.zero_()
                    _lib.call("dc_conv_gemm", C.byref(ds[0]), torch.cuda.current_stream().cuda_stream)
                    torch.cuda.synchronize()
                except _lib.DCError:
                    continue
                err = ((y.float() - ref).norm() / ref.norm()).item()
                t = timed(ds, args.reps)
                flag = " *" if t < best[0] else ""
                if t < best[0]:
                    best = (t, (a, s))
                print(f"    ({a:2d},{s:2d}) {t:7.1f} us  {flops / t / 1e6:6.1f} TF/s  {wbytes / t / 1e3:7.1f} GB/s  "
                      f"err {err:.1e}{flag}", flush=True)
        print(f"  best {best[1]} {best[0]:.1f} us ({t0 / best[0]:.2f}x)", flush=True)


if __name__ == "__main__":
    main()

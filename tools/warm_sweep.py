"""Warm-cache (algo, split) sweep of chosen conv shapes inside a hipGraph (GPU).

The committed table is tuned cold (caches flushed per call), which prices the weight stream as the
sampler step sees it; for shapes whose operands are small and were just written by the previous launch
(TAESD's 64-channel convs, the 1x1 linears) the step runs them L2-warm.  This times every candidate as
20 back-to-back launches captured in one graph and prints the best against the table's choice.
Usage: python tools/warm_sweep.py [--shapes nb,h,w,cin,cout,k ...]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import _lib, ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

DEFAULT = ["1,72,96,64,64,3", "1,144,192,64,64,3", "1,288,384,64,64,3", "1,6,12,1280,1280,1",
           "1,72,96,320,320,1", "1,36,48,640,640,1", "1,18,24,1280,1280,1"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=DEFAULT)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    nalg = _lib.load().dc_conv_num_algos()
    for sh in a.shapes:
        nb, h, w, cin, cout, k = map(int, sh.split(","))
        x = torch.randn(nb * h * w, cin, device=dev).to(torch.bfloat16)
        ktot = -(-(k * k * cin) // 64) * 64
        wt = (torch.randn(cout, ktot, device=dev) / math.sqrt(k * k * cin)).to(torch.bfloat16)
        y = torch.empty(nb * h * w, cout, device=dev, dtype=torch.bfloat16)
        kw = dict(nb=nb, hin=h, win=w, cin=cin, hout=h, wout=w, cout=cout, kh=k, kw=k, pad=k // 2, y=y)
        res = []
        cands = [(None, None)] + [(al, s) for al in range(1, nalg + 1) for s in (1, 2, 4, 8, -1, -2)]
        for al, s in cands:
            try:
                ops.conv_gemm(ctx, x, wt, algo=al, nsplit=s, **kw)
                torch.cuda.synchronize()
            except _lib.DCError:
                continue
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                with torch.cuda.graph(g, stream=st):
                    for _ in range(20):
                        ops.conv_gemm(ctx, x, wt, algo=al, nsplit=s, **kw)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res.append((e0.elapsed_time(e1) / 60 * 1e3, al, s))
        table = [r for r in res if r[1] is None][0]
        best = sorted(r for r in res if r[1] is not None)[:3]
        print(f"{sh}: table {table[0]:.2f} us | best " + ", ".join(f"({al},{s}) {t:.2f}" for t, al, s in best),
              flush=True)


if __name__ == "__main__":
    main()

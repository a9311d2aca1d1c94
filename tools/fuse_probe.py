"""Probe: FF2 + proj_out of the UNet transformer blocks as two GEMMs vs one (GPU, timing only, random operands).

Forward: r3 = gg W2^T + b2 + r2; out = r3 Wp^T + bp + x  (two launches)  vs  out = [gg | r2] [Wp W2 | Wp]^T + b' + x
(one two-source launch, K = 5C).  Backward: dr3 = dout Wp; df = GEGLU'(dr3 W2) (two launches)  vs  one GEMM with
N = 5C (the GEGLU-backward columns timed as plain columns: an upper bound of the fused form's cost).
Each sequence is timed between HIP events after a 512 MiB write (L2 and the Infinity Cache flushed, as the weights are
in the step), best of --reps; shapes missing from the tuned table are autotuned in that cache state first.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, ".")
os.environ.setdefault("DC_TUNE_COLD", "2")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=7)
args = ap.parse_args()
dev = torch.device("cuda:0")
ctx = Ctx(dev, tune=True)
flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
B = torch.bfloat16


def r(*s):
    return (torch.randn(*s, device=dev) * 0.05).to(B)


def timed(fn):
    best = 1e9
    for _ in range(args.reps):
        flush.fill_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best * 1e3


for C, P in ((320, 6912), (640, 1728), (1280, 432)):
    gg, r2, x, dout = r(P, 4 * C), r(P, C), r(P, C), r(P, C)
    w2, wp, wcat = r(C, 4 * C), r(C, C), r(C, 5 * C)
    b2, bp = torch.randn(C, device=dev), torch.randn(C, device=dev)
    r3, out = torch.empty(P, C, dtype=B, device=dev), torch.empty(P, C, dtype=B, device=dev)
    wpt, w2t, wcatt = r(C, C), r(4 * C, C), r(5 * C, C)
    f8, df, dr3, dcat = r(P, 8 * C), torch.empty(P, 8 * C, dtype=B, device=dev), torch.empty(P, C, dtype=B, device=dev), \
        torch.empty(P, 5 * C, dtype=B, device=dev)

    def fwd_a():
        ops.linear(ctx, gg, w2, P, C, r3, bias=b2, resid=r2)
        ops.linear(ctx, r3, wp, P, C, out, bias=bp, resid=x)

    def fwd_b():
        ops.conv_gemm(ctx, gg, wcat, nb=1, hin=1, win=P, cin=5 * C, hout=1, wout=P, cout=C, kh=1, kw=1, pad=0,
                      x2=r2, c1=4 * C, bias=bp, resid=x, y=out)

    def bwd_a():
        ops.linear(ctx, dout, wpt, P, C, dr3)
        ops.linear(ctx, dr3, w2t, P, 4 * C, df, geglu=2, aux=f8)

    def bwd_b():
        ops.linear(ctx, dout, wcatt, P, 5 * C, dcat)

    for f in (fwd_a, fwd_b, bwd_a, bwd_b):   # autotune / warm up
        f()
    torch.cuda.synchronize()
    res = {f.__name__: timed(f) for f in (fwd_a, fwd_b, bwd_a, bwd_b)}
    print(f"C={C} P={P}: fwd two launches {res['fwd_a']:.1f} us, folded {res['fwd_b']:.1f} us | "
          f"bwd two launches {res['bwd_a']:.1f} us, one N=5C launch {res['bwd_b']:.1f} us", flush=True)

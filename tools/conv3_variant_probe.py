"""Probe (GPU, timing only): the level-0 / level-1 3x3 convs of the C2 step over halo and skinny variants (plain
epilogue + residual), one call after a 512 MiB flush (the step's cold-weight regime), best of --reps.  Whether the
weight-streaming skinny form (weights straight into VGPRs, one barrier per input-chunk group) beats the halo tiles
(one barrier per tap) on the large-M levels it was never tuned for."""
import argparse
import math
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402
from depth_completion_amd.weights import pack_conv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
dev = torch.device("cuda:0")
ctx = Ctx(dev)
flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
B = torch.bfloat16


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


VARIANTS = [(33, 1), (31, 1), (31, 3), (62, 1), (63, 1), (64, 1), (43, 1), (44, 1), (45, 1), (46, 1), (47, 1), (45, -2),
            (46, -2), (47, -2), (44, -2), (43, -2)]
for h, w, cin, cout in [(72, 96, 320, 320), (72, 96, 640, 320), (36, 48, 640, 640), (36, 48, 1280, 640)]:
    x = (torch.randn(h * w, cin, device=dev) * 0.1).to(B)
    wt = pack_conv(torch.randn(cout, cin, 3, 3) / math.sqrt(9 * cin)).to(dev, B)
    res = (torch.randn(h * w, cout, device=dev) * 0.1).to(B)
    y = torch.empty(h * w, cout, dtype=B, device=dev)
    out = []
    for algo, ns in VARIANTS:
        try:
            t = timed(lambda: ops.conv_gemm(ctx, x, wt, nb=1, hin=h, win=w, cin=cin, hout=h, wout=w, cout=cout,
                                            resid=res, y=y, algo=algo, nsplit=ns))
            out.append(f"{algo}/{ns}: {t:.1f}")
        except Exception:
            out.append(f"{algo}/{ns}: -")
    print(f"{h}x{w} {cin}->{cout}: " + "  ".join(out), flush=True)

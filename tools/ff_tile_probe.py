"""Probe (GPU, timing only): the transformer FF linears of the C2 step (FF1 with its GEGLU epilogue, the folded FF2 /
proj_out input-gradient with the column-split GEGLU backward) over the im2col tile variants, each call after a 512 MiB
write (L2 and the Infinity Cache flushed, the step's cold-weight regime), best of --reps.  Which tile shape the
short-K, wide-N launches want: per-CU operand fill falls with the tile's area, occupancy with its registers."""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--algos", type=int, nargs="+", default=[1, 3, 5, 10, 11, 12, 13, 14, 15, 16, 20, 21])
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


def r(*s):
    return (torch.randn(*s, device=dev) * 0.05).to(B)


for C, P in ((320, 6912), (640, 1728), (1280, 432)):
    x = r(P, C)
    w1 = r(8 * C, C)
    b1 = torch.randn(8 * C, device=dev)
    f8 = torch.empty(P, 8 * C, dtype=B, device=dev)
    gg = torch.empty(P, 4 * C, dtype=B, device=dev)
    dout, wd = r(P, C), r(5 * C, C)
    df, dr2 = torch.empty(P, 8 * C, dtype=B, device=dev), torch.empty(P, C, dtype=B, device=dev)
    aux = r(P, 8 * C)
    line = []
    for algo in args.algos:
        try:
            t1 = timed(lambda: ops.linear(ctx, x, w1, P, 8 * C, f8, bias=b1, geglu=1, y2=gg, algo=algo, nsplit=1))
            t2 = timed(lambda: ops.linear(ctx, dout, wd, P, 5 * C, df, geglu=2, aux=aux, y2=dr2, geglu_n=4 * C,
                                          algo=algo, nsplit=1))
            line.append(f"{algo}: {t1:.1f}/{t2:.1f}")
        except Exception as e:   # a variant outside its contract
            line.append(f"{algo}: -")
    print(f"C={C} P={P} (FF1 / fold-bwd us): " + "  ".join(line), flush=True)

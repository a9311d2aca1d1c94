"""Run one conv shape with a given (algo, split) N times (for PMC counter runs)."""
import argparse
import math
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="1,72,96,320,320,3")   # nb,h,w,cin,cout,k
ap.add_argument("--algo", type=int, default=12)
ap.add_argument("--split", type=int, default=1)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
nb, h, w, cin, cout, k = map(int, a.shape.split(","))
dev = torch.device("cuda:0")
ctx = Ctx(dev)
x = torch.randn(nb * h * w, cin, device=dev).to(torch.bfloat16)
ktot = -(-(k * k * cin) // 64) * 64
wt = (torch.randn(cout, ktot, device=dev) / math.sqrt(k * k * cin)).to(torch.bfloat16)
y = torch.empty(nb * h * w, cout, device=dev, dtype=torch.bfloat16)
for _ in range(a.reps):
    ops.conv_gemm(ctx, x, wt, nb=nb, hin=h, win=w, cin=cin, hout=h, wout=w, cout=cout, kh=k, kw=k, pad=k // 2, y=y,
                  algo=a.algo, nsplit=a.split)
torch.cuda.synchronize()

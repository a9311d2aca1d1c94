"""Attention fwd/bwd microbenchmark at the UNet shapes (GPU). DC_ATTN_CFG=<i> forces a block configuration.

A/B between two builds: run it once per library with DC_LIB=<path to libdcamd.so> (tools/ab/lib_ab.sh), alternating.
Per shape: forward, and dQ + dK/dV (the backward), best of --reps timed loops of 10 calls each.
"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--no-bwd", action="store_true")
args = ap.parse_args()
dev = torch.device("cuda:0")
ctx = Ctx(dev)


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for n, t, heads in [(1, 6912, 5), (1, 1728, 10), (1, 432, 20), (1, 108, 20), (8, 6912, 5), (8, 1728, 10), (8, 432, 20)]:
    C = heads * 64
    qkv = (torch.randn(n * t, 3 * C, device=dev)).to(torch.bfloat16)
    o = torch.empty(n * t, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(n, heads, t, device=dev)
    do = torch.randn(n * t, C, device=dev).to(torch.bfloat16)
    dq = torch.empty_like(qkv)
    delta = torch.empty(2, n, heads, t, device=dev)
    f = 4.0 * n * t * t * 64 * heads
    fw = [timed(lambda: ops.attn_fwd(ctx, qkv, n, t, heads, o, lse)) for _ in range(args.reps)]
    ms = min(fw)
    print(f"n={n} T={t} H={heads} fwd: {ms*1e3:.1f} us  {f/ms/1e9:.0f} TF/s  (all: {' '.join(f'{x*1e3:.1f}' for x in fw)})",
          flush=True)
    if not args.no_bwd:
        bw = [timed(lambda: ops.attn_bwd(ctx, qkv, o, do, lse, n, t, heads, delta, dq)) for _ in range(args.reps)]
        ms = min(bw)
        print(f"n={n} T={t} H={heads} bwd: {ms*1e3:.1f} us  {3.5*f/ms/1e9:.0f} TF/s (algorithmic incl. recompute)"
              f"  (all: {' '.join(f'{x*1e3:.1f}' for x in bw)})", flush=True)

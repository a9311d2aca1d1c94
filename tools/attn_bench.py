"""Attention fwd/bwd microbenchmark at the UNet shapes (GPU). DC_ATTN_CFG=<i> forces a block configuration.

The forward / backward are timed with the ping-pong forward / backward kernels off and on (DC_ATTN_PP, DC_ATTN_PP_DQ + DC_ATTN_PP_DKDV = 0 / 2 (forced wherever it fits),
alternating, `--reps` pairs)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--no-bwd", action="store_true")
ap.add_argument("--env", default="DC_ATTN_PP", help="forward A/B switch (0 vs 2): DC_ATTN_PP or DC_ATTN_FASTSM")
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


for n, t, heads in [(1, 6912, 5), (1, 1728, 10), (1, 432, 20), (8, 6912, 5), (8, 1728, 10)]:
    C = heads * 64
    qkv = (torch.randn(n * t, 3 * C, device=dev)).to(torch.bfloat16)
    o = torch.empty(n * t, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(n, heads, t, device=dev)
    do = torch.randn(n * t, C, device=dev).to(torch.bfloat16)
    dq = torch.empty_like(qkv)
    delta = torch.empty(n, heads, t, device=dev)
    f = 4.0 * n * t * t * 64 * heads
    res = {"0": [], "2": []}
    for _ in range(args.reps):
        for mode in ("0", "2"):
            os.environ[args.env] = mode
            res[mode].append(timed(lambda: ops.attn_fwd(ctx, qkv, n, t, heads, o, lse)))
    for mode, name in (("0", "fwd"), ("2", f"fwd-{args.env}")):
        ms = min(res[mode])
        print(f"n={n} T={t} H={heads} {name}: {ms*1e3:.1f} us  {f/ms/1e9:.0f} TF/s  (all: "
              f"{' '.join(f'{x*1e3:.1f}' for x in res[mode])})", flush=True)
    if not args.no_bwd:
        rb = {"0": [], "2": []}
        for _ in range(args.reps):
            for mode in ("0", "2"):
                os.environ["DC_ATTN_PP_DQ"] = mode
                os.environ["DC_ATTN_PP_DKDV"] = mode
                rb[mode].append(timed(lambda: ops.attn_bwd(ctx, qkv, o, do, lse, n, t, heads, delta, dq)))
        for mode, name in (("0", "bwd"), ("2", "bwd-pp")):
            ms = min(rb[mode])
            print(f"n={n} T={t} H={heads} {name}: {ms*1e3:.1f} us  {3.5*f/ms/1e9:.0f} TF/s (algorithmic incl. recompute)"
                  f"  (all: {' '.join(f'{x*1e3:.1f}' for x in rb[mode])})", flush=True)

"""Folded cross-attention fwd/bwd timing at the UNet shapes (GPU): 20 launches in a hipGraph between HIP events."""
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

dev = torch.device("cuda:0")
ctx = Ctx(dev)
for rows, c, heads in [(6912, 320, 5), (1728, 640, 10), (432, 1280, 20), (108, 1280, 20), (55296, 320, 5)]:
    x = torch.randn(rows, c, device=dev).to(torch.bfloat16)
    g, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    U, D, c0 = torch.randn(heads, c, device=dev) * 0.05, torch.randn(heads, c, device=dev) * 0.05, torch.zeros(c, device=dev)
    tabs = ops.crossattn_tables(ctx, U, D, heads, c)
    y = torch.empty_like(x)
    st = torch.empty(rows, 2, device=dev)
    pr = torch.empty(rows, heads, device=dev)
    dy = torch.randn_like(x)
    dx = torch.empty_like(x)
    for name, fn in [("fwd", lambda: ops.crossattn_fwd(ctx, x, rows, c, heads, 1e-5, g, b, tabs, c0, y, st, pr)),
                     ("bwd", lambda: ops.crossattn_bwd(ctx, x, rows, c, heads, g, tabs, st, pr, dy, dx))]:
        fn()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(20):
                fn()
        gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"rows={rows} C={c} H={heads} {name}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)

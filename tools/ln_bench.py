"""LayerNorm forward / backward launch times at the UNet token shapes (GPU): 20 launches in a hipGraph between HIP events.
Run once per library build (DC_LIB) to compare."""
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

dev = torch.device("cuda:0")
ctx = Ctx(dev)
for rows, c in [(6912, 320), (1728, 640), (432, 1280), (108, 1280)]:
    x = torch.randn(rows, c, device=dev).to(torch.bfloat16)
    g, b = 1 + 0.1 * torch.randn(c, device=dev), 0.1 * torch.randn(c, device=dev)
    y = torch.empty_like(x)
    st = torch.empty(rows, 2, device=dev)
    dy, add, dx = torch.randn_like(x), torch.randn_like(x), torch.empty_like(x)
    for name, fn in [("fwd", lambda: ops.layernorm(ctx, x, rows, c, g, b, 1e-5, y, st)),
                     ("bwd", lambda: ops.layernorm_bwd(ctx, x, rows, c, None, st, dy, dx, add=add))]:
        fn()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(20):
                fn()
        gr.replay()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
        print(f"rows={rows} C={c} {name}: {best:.1f} us", flush=True)

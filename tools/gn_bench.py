"""GroupNorm(+SiLU) fwd / bwd timing at the UNet shapes (GPU), single-launch (group) and 3-launch forms."""
import os
import sys
import torch
sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402
dev = torch.device("cuda:0"); ctx = Ctx(dev)
shapes = [(1, 6912, 320), (1, 6912, 640), (1, 6912, 960), (1, 1728, 640), (1, 1728, 1280), (1, 1728, 1920),
          (1, 432, 1280), (1, 432, 2560), (1, 108, 1280), (1, 108, 2560), (8, 6912, 320), (8, 432, 1280)]
for (nb, hw, c), path in [(sh, p) for sh in shapes for p in ("3pass", "group")]:
    os.environ["DC_GN_GROUP"] = "0" if path == "3pass" else "-1"
    x = torch.randn(nb * hw, c, device=dev).to(torch.bfloat16)
    g, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    y = torch.empty_like(x); st = torch.empty(nb, 32, 2, device=dev); dy = torch.randn_like(x); dx = torch.empty_like(x)
    for name, fn in [("fwd", lambda: ops.groupnorm(ctx, x, nb, hw, c, g, b, 1e-5, True, y, st)),
                     ("bwd", lambda: ops.groupnorm_bwd(ctx, x, nb, hw, c, g, b, True, st, dy, dx))]:
        for _ in range(3): fn()
        torch.cuda.synchronize()
        # 20 calls captured in one graph: device time per call without the host launch path
        g_ = torch.cuda.CUDAGraph()
        s_ = torch.cuda.Stream()
        with torch.cuda.stream(s_):
            with torch.cuda.graph(g_, stream=s_):
                for _ in range(20): fn()
        g_.replay(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5): g_.replay()
        e1.record(); torch.cuda.synchronize()
        print(f"nb={nb} hw={hw} C={c} {path:5s} {name}: {e0.elapsed_time(e1) / 100 * 1e3:.1f} us (graph)", flush=True)

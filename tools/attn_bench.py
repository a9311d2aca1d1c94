"""Attention fwd/bwd microbenchmark at the UNet shapes (GPU). DC_ATTN_CFG=<i> forces a block configuration."""
import sys, torch
sys.path.insert(0, ".")
from depth_completion_amd import ops
from depth_completion_amd.ops import Ctx
dev = torch.device("cuda:0"); ctx = Ctx(dev)
for n, t, heads in [(1, 6912, 5), (1, 1728, 10), (1, 432, 20), (8, 6912, 5), (8, 1728, 10)]:
    C = heads * 64
    qkv = (torch.randn(n * t, 3 * C, device=dev)).to(torch.bfloat16)
    o = torch.empty(n * t, C, dtype=torch.bfloat16, device=dev); lse = torch.empty(n, heads, t, device=dev)
    do = torch.randn(n * t, C, device=dev).to(torch.bfloat16); dq = torch.empty_like(qkv); delta = torch.empty(n, heads, t, device=dev)
    f = 4.0 * n * t * t * 64 * heads
    for name, fn in [("fwd", lambda: ops.attn_fwd(ctx, qkv, n, t, heads, o, lse)),
                     ("bwd", lambda: ops.attn_bwd(ctx, qkv, o, do, lse, n, t, heads, delta, dq))]:
        for _ in range(3): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): fn()
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        ff = f if name == "fwd" else 3.5 * f
        print(f"n={n} T={t} H={heads} {name}: {ms*1e3:.1f} us  {ff/ms/1e9:.0f} TF/s (algorithmic{' incl. recompute' if name=='bwd' else ''})", flush=True)

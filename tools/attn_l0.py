"""L0 self-attention (T=6912, 5 heads) fwd + bwd, a few launches each (GPU; for PMC passes)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402
dev = torch.device("cuda:0"); ctx = Ctx(dev)
n, t, heads = 1, 6912, 5
C = heads * 64
qkv = torch.randn(n * t, 3 * C, device=dev).to(torch.bfloat16)
o = torch.empty(n * t, C, dtype=torch.bfloat16, device=dev); lse = torch.empty(n, heads, t, device=dev)
do = torch.randn(n * t, C, device=dev).to(torch.bfloat16); dq = torch.empty_like(qkv); delta = torch.empty(n, heads, t, device=dev)
for _ in range(3):
    ops.attn_fwd(ctx, qkv, n, t, heads, o, lse)
    ops.attn_bwd(ctx, qkv, o, do, lse, n, t, heads, delta, dq)
torch.cuda.synchronize()
print("done")

"""Repeatability probe of dc_attn_fwd on one shape (GPU): runs it N times on the same inputs, reports where the
outputs differ (rows, heads, magnitude) and each run's error against fp32 SDPA.
python tools/attn_repeat_probe.py --n 1 --t 1000 --heads 5 --peak 6 [--cfg 1]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1)
ap.add_argument("--t", type=int, default=1000)
ap.add_argument("--heads", type=int, default=5)
ap.add_argument("--peak", type=float, default=6.0)
ap.add_argument("--runs", type=int, default=6)
ap.add_argument("--cfg", default=None)
a = ap.parse_args()
if a.cfg is not None:
    os.environ["DC_ATTN_CFG"] = a.cfg
dev = torch.device("cuda:0")
ctx = Ctx(dev)
n, t, heads = a.n, a.t, a.heads
C = heads * 64
g = torch.Generator().manual_seed(41)
qkv = torch.randn(n, t, 3 * C, generator=g).to(torch.bfloat16).float()
qkv[..., :C] *= a.peak
qkv = qkv.to(torch.bfloat16).float().to(dev)
q, k, v = qkv.split(C, -1)
sh = lambda z: z.view(n, t, heads, 64).transpose(1, 2)  # noqa: E731
ref = F.scaled_dot_product_attention(sh(q), sh(k), sh(v)).transpose(1, 2).reshape(n * t, C)
qkv_b = qkv.to(torch.bfloat16).reshape(n * t, 3 * C).contiguous()
outs = []
for r in range(a.runs):
    ob = torch.zeros(n * t, C, dtype=torch.bfloat16, device=dev)
    lse = torch.zeros(n, heads, t, device=dev)
    ops.attn_fwd(ctx, qkv_b, n, t, heads, ob, lse)
    torch.cuda.synchronize()
    outs.append((ob.float(), lse))
    err = float((ob.float() - ref).norm() / ref.norm())
    print(f"run {r}: rel err vs SDPA {err:.3e}")
for r in range(1, a.runs):
    d = (outs[r][0] - outs[0][0]).abs()
    dl = (outs[r][1] - outs[0][1]).abs()
    rows = torch.nonzero(d.amax(1) > 0).flatten()
    print(f"run {r} vs 0: O max diff {float(d.max()):.3e} in {rows.numel()} rows "
          f"{rows[:12].tolist()} heads {sorted(set((torch.nonzero(d > 0)[:, 1] // 64).tolist()))[:10]}; "
          f"lse max diff {float(dl.max()):.3e} at {torch.nonzero(dl > 0)[:6].tolist()}")

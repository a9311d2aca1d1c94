"""Attention forward accuracy vs fp32 SDPA at the UNet shapes (GPU): relative error of O and of the LSE, for
unit-scale and peaked (3x) scores.  DC_LIB=<path> selects another build (A/B)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

dev = torch.device("cuda:0")
ctx = Ctx(dev)
for n, t, heads in [(1, 6912, 5), (1, 1728, 10), (1, 432, 20), (2, 1000, 3)]:
    for scale in (1.0, 3.0):
        C = heads * 64
        g = torch.Generator(device=dev).manual_seed(5)
        qkv = (torch.randn(n * t, 3 * C, device=dev, generator=g) * scale).to(torch.bfloat16)
        q, k, v = qkv.float().view(n, t, 3 * C).split(C, -1)
        sh = lambda z: z.reshape(n, t, heads, 64).transpose(1, 2)  # noqa: E731
        ref = F.scaled_dot_product_attention(sh(q), sh(k), sh(v)).transpose(1, 2).reshape(n * t, C)
        lse_ref = torch.logsumexp(torch.einsum("nhqd,nhkd->nhqk", sh(q), sh(k)) / 8, -1)
        o = torch.empty(n * t, C, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(n, heads, t, device=dev)
        ops.attn_fwd(ctx, qkv, n, t, heads, o, lse)
        torch.cuda.synchronize()
        eo = float((o.float() - ref).norm() / ref.norm())
        el = float((lse - lse_ref).abs().max())
        # bf16 rounding of the fp32 reference itself: the floor any bf16 output sits on
        floor = float((ref.to(torch.bfloat16).float() - ref).norm() / ref.norm())
        print(f"n={n} T={t} H={heads} scale={scale}: O rel {eo:.3e} (bf16 floor {floor:.3e})  LSE max abs {el:.3e}",
              flush=True)

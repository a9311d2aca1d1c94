"""Fused vs separate GroupNorm statistics on one UNet forward + backward (GPU): every plan buffer compared in
allocation order, to find the first one that departs beyond rounding (tools, not a test).

    python tools/gn_fuse_diff.py [--cfg tiny|full] [--n 2 --h 16 --w 16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="tiny")
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--h", type=int, default=16)
    ap.add_argument("--w", type=int, default=16)
    a = ap.parse_args()
    from depth_completion_amd import synthetic
    from depth_completion_amd.config import MARIGOLD_V1, TINY
    from depth_completion_amd.ops import Ctx
    from depth_completion_amd.unet import UNetHIP
    dev = torch.device("cuda:0")
    cfg = TINY if a.cfg == "tiny" else MARIGOLD_V1
    ctx = Ctx(dev)
    sd = synthetic.unet_state_dict(cfg, 11)
    emb = synthetic.text_embedding(13, cfg.cross_attention_dim)
    net = UNetHIP({k: v.float() for k, v in sd.items()}, cfg, dev, emb)
    net.build_temb_tables(ctx, torch.tensor([999]))
    ctx.step.zero_()
    g = torch.Generator().manual_seed(1)
    plans = []
    for fuse in ("1", "0"):
        os.environ["DC_GN_FUSE"] = fuse
        p = net.plan(ctx, a.n, a.h, a.w)
        p.x8.copy_(torch.randn(p.x8.shape, generator=g).to(torch.bfloat16).to(dev) if not plans else plans[0].x8)
        p.dv.copy_(torch.randn(p.dv.shape, generator=g).to(torch.bfloat16).to(dev) if not plans else plans[0].dv)
        p.forward()
        p.backward()
        plans.append(p)
    torch.cuda.synchronize()
    f, s = plans
    print(f"{len(f.saved)} buffers")
    for i, (x, y) in enumerate(zip(f.saved, s.saved)):
        if x.shape != y.shape or x.dtype != y.dtype or x.dtype == torch.int64:
            continue
        d = (x.float() - y.float()).norm() / (y.float().norm() + 1e-20)
        if d > 1e-3:
            print(f"buffer {i} {tuple(x.shape)} {x.dtype}: rel diff {float(d):.4g}")


if __name__ == "__main__":
    main()

"""Layer-by-layer comparison of the HIP UNet plan against the oracle (debug helper, GPU)."""
import sys
import torch
sys.path.insert(0, ".")
from oracle.diffusers_ref import (UNet2DConditionModel, synthetic_state_dict, synthetic_text_embedding,
                                  tiny_unet_config, ResnetBlock2D, Transformer2DModel, Downsample2D, Upsample2D)
from depth_completion_amd.config import TINY
from depth_completion_amd.unet import UNetHIP
from depth_completion_amd.ops import Ctx

dev = torch.device("cuda:0")
def rel(a, b): return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))

def run(n, h, w, same=False):
    ocfg = tiny_unet_config()
    m = UNet2DConditionModel(ocfg); sd = synthetic_state_dict(m, 11); m.load_state_dict(sd)
    m = m.to(torch.bfloat16).float().to(dev)
    emb = synthetic_text_embedding(13, ocfg.cross_attention_dim).to(dev)
    g = torch.Generator().manual_seed(1)
    x8 = torch.randn(1 if same else n, 8, h, w, generator=g).to(torch.bfloat16).float().to(dev)
    if same: x8 = x8.repeat(n, 1, 1, 1)
    outs = []
    hooks = [mod.register_forward_hook(lambda mod, i, o: outs.append((type(mod).__name__, o)))
             for mod in m.modules() if isinstance(mod, (ResnetBlock2D, Transformer2DModel, Downsample2D, Upsample2D))]
    with torch.no_grad():
        v = m(x8, torch.tensor(999, device=dev), emb)[0]
    ctx = Ctx(dev)
    net = UNetHIP({k: t.float() for k, t in sd.items()}, TINY, dev, emb.cpu())
    net.build_temb_tables(ctx, torch.tensor([999])); ctx.step.zero_()
    plan = net.plan(ctx, n, h, w)
    plan.x8.copy_(x8.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.bfloat16))
    plan.forward(); torch.cuda.synchronize()
    tape = [(k, d) for k, d in plan.tape if k in ("resnet", "transformer", "down", "up")]
    print(f"n={n} {h}x{w} same={same}: {len(tape)} tape vs {len(outs)} oracle")
    for (k, d), (name, o) in zip(tape, outs):
        nn_, c, hh, ww = o.shape
        got = d["out"].float().reshape(nn_, hh, ww, c).permute(0, 3, 1, 2)
        errs = [rel(got[i], o[i]) for i in range(nn_)]
        print(f"  {k:12s} {name:20s} {tuple(o.shape)} err per frame {['%.4f' % e for e in errs]}")
    vh = plan.v[:, :4].float().reshape(n, h, w, 4).permute(0, 3, 1, 2)
    print("  v err per frame", [round(rel(vh[i], v[i]), 4) for i in range(n)])

run(1, 16, 16)
run(2, 16, 16)
run(2, 6, 8)

import sys
import torch
sys.path.insert(0, ".")
from oracle.diffusers_ref import AutoencoderTiny, synthetic_taesd_state_dict
from depth_completion_amd.taesd import TAESDHIP
from depth_completion_amd.ops import Ctx
dev = torch.device("cuda:0")
def rel(a, b): return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))
for n in (1, 2):
    vae = AutoencoderTiny(); sd = synthetic_taesd_state_dict(vae, 12); vae.load_state_dict(sd)
    v32 = vae.to(torch.bfloat16).float().to(dev)
    h, w = 6, 8
    z = torch.randn(n, 4, h, w, generator=torch.Generator().manual_seed(2)).to(torch.bfloat16).float().to(dev)
    zc = (torch.tanh(z / 3) * 3).to(torch.bfloat16).float().detach().requires_grad_(True)
    acts = []
    hooks = [l.register_forward_hook(lambda mod, i, o: acts.append(o)) for l in v32.decoder.layers]
    out = v32.decoder.layers(zc)
    gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16).float().to(dev)
    # grads of each layer output
    grads = [torch.autograd.grad(out, a, gout, retain_graph=True)[0] for a in acts[:-1]]
    gin = torch.autograd.grad(out, zc, gout)[0]
    ctx = Ctx(dev)
    net = TAESDHIP({k: t.float() for k, t in sd.items()}, dev)
    dp = net.decoder_plan(ctx, n, h, w)
    dp.tin.zero_(); dp.tin[:, :4].copy_(zc.detach().permute(0, 2, 3, 1).reshape(-1, 4).to(torch.bfloat16))
    dp.forward(); dp.dout.zero_()
    dp.dout[:, :3].copy_(gout.permute(0, 2, 3, 1).reshape(-1, 3).to(torch.bfloat16))
    dp.backward(); torch.cuda.synchronize()
    H, W = 8*h, 8*w
    print("n", n, "out err", rel(dp.out[:, :3].float().reshape(n, H, W, 3).permute(0, 3, 1, 2), out),
          "gin err", rel(dp.dtin[:, :4].float().reshape(n, h, w, 4).permute(0, 3, 1, 2), gin))
    # per-buffer grads in backward order: compare block input grads
    for i, b in enumerate(dp.saved):
        pass

"""Split-K fixup check: every algo x split against split 1 on a small linear and a 3x3 conv (GPU)."""
import sys, torch
sys.path.insert(0, ".")
from depth_completion_amd import ops, _lib
from depth_completion_amd.ops import Ctx
dev = torch.device("cuda:0"); ctx = Ctx(dev)
nalg = _lib.load().dc_conv_num_algos()
torch.manual_seed(0)
for (M, K, N) in [(180, 1728, 192), (432, 1280, 1280)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    ref = (x.float() @ w.float().t())
    for a in range(1, nalg + 1):
        res = []
        for s in (1, 2, 3, 8):
            y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
            ops.conv_gemm(ctx, x, w, nb=1, hin=1, win=M, cin=K, hout=1, wout=M, cout=N, kh=1, kw=1, pad=0, y=y, algo=a, nsplit=s)
            torch.cuda.synchronize()
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            res.append(f"s{s}:{err:.1e}/{int(torch.isnan(y.float()).sum())}")
        print(M, K, N, "algo", a, " ".join(res), flush=True)

"""Probe (GPU, timing only): the single-launch group GroupNorm (dc_groupnorm_fwd / _bwd, one block per (frame, group))
against the one-pass forms that read producer-accumulated statistics (dc_groupnorm_fwd_acc / _bwd_acc), at the
level-2 / level-3 batch-1 shapes, each call timed inside a 20-call graph (device time without the host path).
The accumulators are zero (values meaningless); only the launch cost is measured.
"""
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

dev = torch.device("cuda:0")
ctx = Ctx(dev)


def graph_time(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


for nb, hw, c in [(1, 432, 640), (1, 432, 1280), (1, 432, 1920), (1, 432, 2560), (1, 108, 1280), (1, 108, 2560),
                  (1, 1728, 640), (1, 6912, 320)]:
    x = torch.randn(nb * hw, c, device=dev).to(torch.bfloat16)
    g, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    y = torch.empty_like(x)
    st = torch.zeros(nb, 32, 2, device=dev)
    st[..., 1] = 1.0
    dy, dx = torch.randn_like(x), torch.empty_like(x)
    acc = torch.zeros(ops.gn_acc_words(nb), dtype=torch.int64, device=dev)
    res = {
        "group fwd": graph_time(lambda: ops.groupnorm(ctx, x, nb, hw, c, g, b, 1e-5, True, y, st)),
        "acc fwd": graph_time(lambda: ops.groupnorm_acc(ctx, x, nb, hw, c, g, b, 1e-5, True, acc, y, st)),
        "group bwd": graph_time(lambda: ops.groupnorm_bwd(ctx, x, nb, hw, c, g, b, True, st, dy, dx)),
        "acc bwd": graph_time(lambda: ops.groupnorm_bwd_acc(ctx, x, nb, hw, c, g, st, acc, dy, dx)),
    }
    print(f"nb={nb} hw={hw} C={c}: " + ", ".join(f"{k} {v:.1f} us" for k, v in res.items()), flush=True)

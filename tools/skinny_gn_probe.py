"""Probe (GPU, timing only): the level-2 / level-3 skinny convs with and without the fused GroupNorm statistics
(dc_gn_fuse modes 1 / 2) in their epilogues, and the diagnostic arms that skip parts of it (DC_HALO_DIAG 8: no
accumulator adds; 16: no block fold either), each call timed inside a 20-call graph.
Args: [skinny | halo | l01] (the level-2 / 3 skinny shapes, level-0 / 1 halo shapes, or level-0 / 1 halo vs skinny)."""
import math
import os
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402
from depth_completion_amd.weights import pack_conv  # noqa: E402

dev = torch.device("cuda:0")
ctx = Ctx(dev)
G = 32


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


def r(*s):
    return (torch.randn(*s, device=dev) * 0.05).to(torch.bfloat16)


SHAPES = {"skinny": [(9, 12, 1280, 43, -10), (9, 12, 1280, 43, 10), (9, 12, 1280, 43, 1), (18, 24, 1280, 47, -4),
                     (18, 24, 640, 47, -4)],
          "halo": [(72, 96, 320, 33, 1), (36, 48, 640, 31, 3), (36, 48, 640, 33, 1), (72, 96, 640, 62, 1)],
          # level-0 / 1: the skinny form against the halo tile it replaced or kept (profiles/r05ag/)
          "l01": [(72, 96, 320, 33, 1), (72, 96, 320, 47, 1), (72, 96, 640, 62, 1), (72, 96, 640, 47, 1),
                  (36, 48, 1280, 31, 5), (36, 48, 1280, 47, 1)]}
for h, w, c, algo, ns in SHAPES[sys.argv[1] if len(sys.argv) > 1 else "skinny"]:
    x = r(h * w, c)
    wt = pack_conv(torch.randn(c, c, 3, 3) / math.sqrt(9 * c)).to(dev, torch.bfloat16)
    res = r(h * w, c)
    y = torch.empty(h * w, c, dtype=torch.bfloat16, device=dev)
    acc = torch.zeros(ops.gn_acc_words(1), dtype=torch.int64, device=dev)
    st = torch.zeros(1, G, 2, device=dev)
    st[..., 1] = 1.0
    gam, bet = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    kw = dict(nb=1, hin=h, win=w, cin=c, hout=h, wout=w, cout=c, resid=res, algo=algo, nsplit=ns)
    g1 = ops.gn_fuse_fwd([(acc, 0, G, c // G, h * w)])
    g2 = ops.gn_fuse_bwd(acc, G, c // G, h * w, x, st, gam, bet, True)
    out = []
    for name, gn, diag in [("plain", None, "0"), ("gn1", g1, "0"), ("gn1 no-adds", g1, "8"),
                           ("gn1 no-fold", g1, "16"), ("gn2", g2, "0"), ("gn2 no-adds", g2, "8")]:
        os.environ["DC_HALO_DIAG"] = diag
        out.append(f"{name} {graph_time(lambda: ops.conv_gemm(ctx, x, wt, y=y, gn=gn, **kw)):.1f}")
    os.environ["DC_HALO_DIAG"] = "0"
    print(f"{h}x{w} C={c} algo {algo} split {ns}: " + ", ".join(out) + " us", flush=True)

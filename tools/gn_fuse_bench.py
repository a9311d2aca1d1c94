"""Cost of the fused GroupNorm-statistics epilogue on the C2 shapes (GPU): each conv timed plain, with mode-1
statistics, with mode-2 (backward) statistics, each with and without the accumulator adds (DC_HALO_DIAG=8 skips
them, 32 stops after the shuffles, 16 after the row loop; experiments only), in a captured graph of 20 launches with L2 flushed before the graph.

    python tools/gn_fuse_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

dev = torch.device("cuda:0")
# (name, nb, h, w, cin, cout, k, algo, split): the L0 / L1 / L2 / L3 resnet convs and the L0 / L2 1x1 linears
SHAPES = [("L0 3x3", 1, 72, 96, 320, 320, 3, 31, 1), ("L1 3x3", 1, 36, 48, 640, 640, 3, 31, 2),
          ("L2 3x3", 1, 18, 24, 1280, 1280, 3, 29, 3), ("L3 3x3", 1, 9, 12, 1280, 1280, 3, 29, 5),
          ("L0 1x1", 1, 1, 6912, 320, 320, 1, 13, 1), ("L2 1x1", 1, 1, 432, 1280, 1280, 1, 3, 2)]


def main():
    from depth_completion_amd import ops
    ctx = ops.Ctx(dev)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for name, nb, h, w, cin, cout, k, algo, split in SHAPES:
        x = torch.randn(nb * h * w, cin, device=dev).to(torch.bfloat16)
        wt = (torch.randn(cout, k * k * cin, device=dev) / (k * k * cin) ** 0.5).to(torch.bfloat16)
        y = torch.empty(nb * h * w, cout, dtype=torch.bfloat16, device=dev)
        acc = torch.zeros(ops.gn_acc_words(nb), dtype=torch.int64, device=dev)
        stats = torch.zeros(nb, 32, 2, device=dev)
        gamma = torch.ones(cout, device=dev)
        beta = torch.zeros(cout, device=dev)
        hw = h * w
        g1 = ops.gn_fuse_fwd([(acc, 0, 32, cout // 32, hw)])
        g2 = ops.gn_fuse_bwd(acc, 32, cout // 32, hw, y, stats, gamma, beta, True)
        kw = dict(nb=nb, hin=h, win=w, cin=cin, hout=h, wout=w, cout=cout, kh=k, kw=k, pad=k // 2, algo=algo,
                  nsplit=split)
        res = []
        for tag, gn, diag in (("plain", None, "0"), ("plain-noepi", None, "64"), ("fwd-noepi", g1, "64"),
                              ("fwd", g1, "0"), ("fwd-noadd", g1, "8"),
                              ("fwd-shfl", g1, "32"), ("fwd-rows", g1, "16"), ("bwd", g2, "0"),
                              ("bwd-noadd", g2, "8"), ("bwd-rows", g2, "16")):
            os.environ["DC_HALO_DIAG"] = diag
            graph = torch.cuda.CUDAGraph()
            ops.conv_gemm(ctx, x, wt, y=y, gn=gn, **kw)
            torch.cuda.synchronize()
            with torch.cuda.graph(graph):
                for _ in range(20):
                    ops.conv_gemm(ctx, x, wt, y=y, gn=gn, **kw)
            best = 1e9
            for _ in range(5):
                flush.fill_(1)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graph.replay()
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
            res.append(f"{tag} {best:6.1f}")
        os.environ["DC_HALO_DIAG"] = "0"
        print(f"{name:8s} algo {algo} split {split}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()

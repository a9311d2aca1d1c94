"""Time the halo-tile direct 3x3 conv variants against the tuned im2col choice on the sampler's 3x3 shapes (GPU).

For each shape: the committed table's (algo, split) and every halo algo x split, each as a hipGraph of `reps`
back-to-back launches between HIP events (warm L2, as tools/conv_breakdown.py), plus the output's relative
error against the tuned launch (a quick correctness screen; tests/test_gpu_kernels.py has the real tests).
Usage: python tools/halo_bench.py [--reps 20] [--set c2|taesd|all]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depth_completion_amd import _lib, ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

# (nb, hin, win, cin, hout, wout, cout, mode)
C2 = [(1, 72, 96, 320, 72, 96, 320, 0), (1, 72, 96, 640, 72, 96, 320, 0), (1, 72, 96, 960, 72, 96, 320, 0),
      (1, 72, 96, 320, 72, 96, 640, 0), (1, 72, 96, 640, 72, 96, 640, 0), (1, 36, 48, 640, 72, 96, 640, 1),
      (1, 36, 48, 640, 36, 48, 640, 0), (1, 36, 48, 1280, 36, 48, 640, 0), (1, 36, 48, 1920, 36, 48, 640, 0),
      (1, 36, 48, 640, 36, 48, 1280, 0), (1, 36, 48, 1280, 36, 48, 1280, 0), (1, 18, 24, 1280, 36, 48, 1280, 1),
      (1, 18, 24, 1280, 18, 24, 1280, 0), (1, 18, 24, 2560, 18, 24, 1280, 0), (1, 18, 24, 1280, 18, 24, 2560, 0),
      (1, 9, 12, 1280, 18, 24, 1280, 1),
      (1, 9, 12, 1280, 9, 12, 1280, 0), (1, 9, 12, 2560, 9, 12, 1280, 0), (1, 9, 12, 1280, 9, 12, 2560, 0),
      (1, 72, 96, 320, 72, 96, 4, 0)]
TAESD = [(1, 72, 96, 64, 72, 96, 64, 0), (1, 72, 96, 64, 144, 192, 64, 1), (1, 144, 192, 64, 144, 192, 64, 0),
         (1, 144, 192, 64, 288, 384, 64, 1), (1, 288, 384, 64, 288, 384, 64, 0), (1, 576, 768, 64, 576, 768, 64, 0),
         (8, 72, 96, 320, 72, 96, 320, 0), (8, 36, 48, 640, 36, 48, 640, 0)]


def run(ctx, d, reps, wts=None):
    """reps launches in one graph; wts: weight copies cycled over the launches (weights cold, as in the step)"""
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            _lib.call("dc_conv_gemm", ctx_desc(d), torch.cuda.current_stream().cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    w0 = d.w
    with torch.cuda.graph(g):
        for i in range(reps):
            if wts:
                d.w = wts[i % len(wts)].data_ptr()
            _lib.call("dc_conv_gemm", ctx_desc(d), torch.cuda.current_stream().cuda_stream)
    d.w = w0
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def ctx_desc(d):
    import ctypes as C
    return C.byref(d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--set", default="all")
    ap.add_argument("--algos", type=int, nargs="*", default=None)
    ap.add_argument("--cold", type=int, default=0, help="weight copies cycled over the launches (0: one, warm)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    nalg = _lib.load().dc_conv_num_algos()
    halo = args.algos or list(range(23, nalg + 1))
    shapes = {"c2": C2, "taesd": TAESD, "all": C2 + TAESD}[args.set]
    for nb, hin, win, cin, hout, wout, cout, mode in shapes:
        x = torch.randn(nb * hin * win, cin, device=dev).to(torch.bfloat16)
        wt = (torch.randn(cout, 9 * cin, device=dev) / math.sqrt(9 * cin)).to(torch.bfloat16)
        b = torch.randn(cout, device=dev)
        ldy = max(8, -(-cout // 8) * 8)
        y0 = torch.zeros(nb * hout * wout, ldy, device=dev, dtype=torch.bfloat16)
        d = ops.conv_desc(ctx, x, wt, nb=nb, hin=hin, win=win, cin=cin, hout=hout, wout=wout, cout=cout, mode=mode,
                          bias=b, y=y0)
        wts = [wt] + [wt.clone() for _ in range(args.cold - 1)] if args.cold > 1 else None
        tuned = (d.algo, d.splitk)
        t0 = run(ctx, d, args.reps, wts)
        ref = y0.clone()
        flops = 2.0 * nb * hout * wout * cout * 9 * cin
        best = (float("inf"), None, 0.0)
        per_algo = {}
        for a in halo:
            for sp in (1, 2, 3, 4, 5, 8, 10, 16):
                if sp > cin // 64:
                    continue
                d.algo, d.splitk = a, sp
                y0.zero_()
                t = run(ctx, d, args.reps, wts)
                err = float((y0.float() - ref.float()).norm() / ref.float().norm())
                if err > 2e-2:
                    print(f"   !! algo {a} split {sp}: rel err {err:.3e}", flush=True)
                if t < best[0]:
                    best = (t, (a, sp), err)
                if t < per_algo.get(a, (float("inf"),))[0]:
                    per_algo[a] = (t, sp)
        print(f"nb={nb} {hin}x{win}->{hout}x{wout} cin={cin} cout={cout} mode={mode}: tuned {tuned} {t0:7.1f} us "
              f"({flops / t0 / 1e6:6.0f} TF/s) | best halo {best[1]} {best[0]:7.1f} us ({flops / best[0] / 1e6:6.0f} "
              f"TF/s, err {best[2]:.1e}) x{t0 / best[0]:.2f}", flush=True)
        top = sorted(per_algo.items(), key=lambda kv: kv[1][0])
        print("      " + "  ".join(f"{a}/{sp}:{t:.1f}" for a, (t, sp) in top), flush=True)


if __name__ == "__main__":
    main()

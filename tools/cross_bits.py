"""Folded cross-attention outputs on seeded inputs, saved for a bitwise comparison of two library builds (GPU).

    DC_LIB=ab/lib_a.so python tools/cross_bits.py out_a.pt ; python tools/cross_bits.py out_b.pt
    python tools/cross_bits.py --compare out_a.pt out_b.pt
Shapes: the UNet levels' (rows, C, heads) plus ragged row counts; forward (y, stats, probs, norm3 stats), backward and
the norm3-fused backward.
"""
import sys

import torch

sys.path.insert(0, ".")

CASES = [(6912, 320, 5), (1728, 640, 10), (432, 1280, 20), (108, 1280, 20), (437, 1280, 20), (101, 320, 5)]


def run(path):
    from depth_completion_amd import ops
    from depth_completion_amd.ops import Ctx
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    out = {}
    for rows, c, heads in CASES:
        g = torch.Generator(device="cpu").manual_seed(rows * 7 + c)
        rn = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
        x = rn(rows, c).to(torch.bfloat16)
        gamma, beta = 1 + 0.1 * rn(c), 0.1 * rn(c)
        U, D, c0 = rn(heads, c) * 0.05, rn(heads, c) * 0.05, 0.1 * rn(c)
        tabs = ops.crossattn_tables(ctx, U, D, heads, c)
        y = torch.empty_like(x)
        st, pr, ys = torch.empty(rows, 2, device=dev), torch.empty(rows, heads, device=dev), torch.empty(rows, 2, device=dev)
        ops.crossattn_fwd(ctx, x, rows, c, heads, 1e-5, gamma, beta, tabs, c0, y, st, pr, ystats=ys, yeps=1e-5)
        dy = rn(rows, c).to(torch.bfloat16)
        dx = torch.empty_like(x)
        ops.crossattn_bwd(ctx, x, rows, c, heads, gamma, tabs, st, pr, dy, dx)
        dl, add = rn(rows, c).to(torch.bfloat16), rn(rows, c).to(torch.bfloat16)
        dx2 = torch.empty_like(x)
        ops.crossattn_bwd_ln(ctx, x, rows, c, heads, gamma, tabs, st, pr, dl, y, ys, add, dx2)
        torch.cuda.synchronize()
        for k, v in dict(y=y, st=st, pr=pr, ys=ys, dx=dx, dx2=dx2).items():
            out[f"{rows}_{c}_{k}"] = v.cpu()
    torch.save(out, path)
    print(f"saved {len(out)} tensors to {path}")


def compare(a, b):
    ta, tb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = [k for k in ta if not torch.equal(ta[k].view(torch.int16) if ta[k].dtype == torch.bfloat16 else ta[k],
                                            tb[k].view(torch.int16) if tb[k].dtype == torch.bfloat16 else tb[k])]
    print(f"{len(ta)} tensors, {len(bad)} differ: {bad}")
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])

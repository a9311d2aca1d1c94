"""GroupNorm statistics fused into the producing conv's epilogue (include/dcamd.h dc_gn_fuse) and the one-pass
GroupNorm kernels that read them (dc_groupnorm_fwd_acc / dc_groupnorm_bwd_acc), against torch fp32 (GPU).

The fused epilogue must store exactly what the plain epilogue stores (bitwise, same variant), the accumulated sums
are exact (statistics within fp64-vs-fp32 rounding of torch's), every result is bitwise reproducible, and the
GroupNorm outputs / input-gradients meet the same bars as the separate-pass kernels (tests/test_gpu_kernels.py).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = torch.device("cuda:0")
G = 32


def rel(a, b):
    a = a.float()
    b = b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from depth_completion_amd.ops import Ctx
    return Ctx(dev)


def nhwc(x):
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c).to(torch.bfloat16).contiguous()


def nchw(t, n, h, w):
    return t.float().reshape(n, h, w, -1).permute(0, 3, 1, 2)


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).float().to(dev)


def acc_for(n, groups=G):
    from depth_completion_amd import ops
    return torch.zeros(ops.gn_acc_words(n, groups), dtype=torch.int64, device=dev)


def group_stats(y, n, hw, c, groups=G):
    """(mean, rstd) per (frame, group) of [n*hw, c] rows, fp64."""
    v = y.double().reshape(n, hw, groups, c // groups).permute(0, 2, 1, 3).reshape(n, groups, -1)
    return v.mean(-1), v.var(-1, unbiased=False)


# conv variants: (algo, nsplit) -- im2col tiles plain / split-K / stream-K, halo tiles plain / split, and the skinny
# halo tiles (43 ..: 9 x 12 / 9 x 24 / 6 x 24 pixels, 64 or 128 channels) plain, last-arriver split (> 0) and
# two-kernel split (< 0, the statistics in skinny_reduce_kernel)
VARIANTS = [(3, 1), (13, 2), (10, 1), (1, -1), (18, 1), (23, 1), (29, 2), (31, 1), (33, 3), (62, 1), (63, 2), (64, 1),
            (43, 1), (44, 2), (45, -2), (46, -2), (47, 1)]


@pytest.mark.parametrize("algo,nsplit", VARIANTS)
def test_fused_forward_stats(ctx, algo, nsplit):
    """3x3 conv (bias + residual) with mode-1 statistics: the stored output equals the plain epilogue's bitwise,
    the accumulated statistics match fp64 torch on the stored values, and GN(+SiLU) from them matches torch."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    n, cin, cout, h, w = 2, 128, 320, 12, 20
    x = nhwc(rnd(n, cin, h, w, seed=1))
    wt = pack_conv(rnd(cout, cin, 3, 3, scale=1 / math.sqrt(9 * cin), seed=2)).to(dev, torch.bfloat16)
    b = rnd(cout, seed=3)
    res = nhwc(rnd(n, cout, h, w, seed=4) + 0.7)
    kw = dict(nb=n, hin=h, win=w, cin=cin, hout=h, wout=w, cout=cout, bias=b, resid=res, algo=algo, nsplit=nsplit)
    y0 = torch.empty(n * h * w, cout, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, x, wt, y=y0, **kw)
    acc = acc_for(n)
    y = torch.empty_like(y0)
    g = ops.gn_fuse_fwd([(acc, 0, G, cout // G, h * w)])
    ops.conv_gemm(ctx, x, wt, y=y, gn=g, **kw)
    gamma = (1 + 0.1 * rnd(cout, seed=5)).to(torch.bfloat16).float()
    beta = (0.1 * rnd(cout, seed=6)).to(torch.bfloat16).float()
    out = torch.empty_like(y)
    stats = torch.empty(n, G, 2, device=dev)
    ops.groupnorm_acc(ctx, y, n, h * w, cout, gamma, beta, 1e-5, True, acc, out, stats)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    mean, var = group_stats(y, n, h * w, cout)
    assert rel(stats[..., 0], mean) < 1e-6
    assert rel(stats[..., 1], (var + 1e-5).rsqrt()) < 1e-6
    ref = F.silu(F.group_norm(nchw(y, n, h, w), G, gamma, beta, eps=1e-5))
    assert rel(nchw(out, n, h, w), ref) < 1e-2


def test_fused_concat_two_producers(ctx):
    """An up-block concat: x (640 channels) and the skip (320) come from two convs adding into one accumulator;
    groups of 30 channels straddle the boundary (group 21 has channels of both).  The skip's producer also feeds
    a direct GroupNorm of its own (two targets)."""
    from depth_completion_amd import ops
    n, h, w, ca, cb = 2, 9, 12, 640, 320
    c = ca + cb
    xa_in, xb_in = nhwc(rnd(n, 64, h, w, seed=7)), nhwc(rnd(n, 64, h, w, seed=8))
    wa = rnd(ca, 64, scale=0.2, seed=9).to(torch.bfloat16)
    wb = rnd(cb, 64, scale=0.2, seed=10).to(torch.bfloat16)
    acc_cat, acc_b = acc_for(n), acc_for(n)
    xa = torch.empty(n * h * w, ca, dtype=torch.bfloat16, device=dev)
    xb = torch.empty(n * h * w, cb, dtype=torch.bfloat16, device=dev)
    ops.linear(ctx, xa_in, wa, n * h * w, ca, xa, gn=ops.gn_fuse_fwd([(acc_cat, 0, G, c // G, h * w)]))
    ops.linear(ctx, xb_in, wb, n * h * w, cb, xb,
               gn=ops.gn_fuse_fwd([(acc_b, 0, G, cb // G, h * w), (acc_cat, ca, G, c // G, h * w)]))
    gamma = (1 + 0.1 * rnd(c, seed=11)).to(torch.bfloat16).float()
    beta = (0.1 * rnd(c, seed=12)).to(torch.bfloat16).float()
    y = torch.empty(n * h * w, c, dtype=torch.bfloat16, device=dev)
    st = torch.empty(n, G, 2, device=dev)
    ops.groupnorm_acc(ctx, xa, n, h * w, c, gamma, beta, 1e-5, True, acc_cat, y, st, x2=xb, c1=ca)
    yb = torch.empty_like(xb)
    stb = torch.empty(n, G, 2, device=dev)
    ops.groupnorm_acc(ctx, xb, n, h * w, cb, gamma[:cb], beta[:cb], 1e-5, False, acc_b, yb, stb)
    torch.cuda.synchronize()
    cat = torch.cat([xa, xb], 1)
    mean, var = group_stats(cat, n, h * w, c)
    assert rel(st[..., 0], mean) < 1e-6 and rel(st[..., 1], (var + 1e-5).rsqrt()) < 1e-6
    ref = F.silu(F.group_norm(nchw(cat, n, h, w), G, gamma, beta, eps=1e-5))
    assert rel(nchw(y, n, h, w), ref) < 1e-2
    refb = F.group_norm(nchw(xb, n, h, w), G, gamma[:cb], beta[:cb], eps=1e-5)
    assert rel(nchw(yb, n, h, w), refb) < 1e-2


@pytest.mark.parametrize("n,t,c,algo,nsplit", [(3, 108, 320, 3, 1), (8, 432, 1280, 10, 1), (3, 108, 64, 13, 1),
                                               (5, 36, 640, 0, 0), (3, 108, 320, 49, 1), (3, 108, 320, 49, -2),
                                               (8, 432, 1280, 53, 1), (5, 36, 640, 51, 2), (5, 36, 640, 52, -2)])
def test_fused_linear_frames_straddle(ctx, n, t, c, algo, nsplit):
    """A linear over n * T token rows (T not a multiple of the tile's wave rows): waves whose rows straddle two
    frames add per row; per-frame statistics exact, results bitwise repeatable.  The skinny row tiles (49 ..: 112 /
    224 / 64 rows) straddle frames in their own epilogue and in skinny_reduce_kernel's 16-row fragments."""
    from depth_completion_amd import ops
    k = 256
    a = rnd(n * t, k, seed=13).to(torch.bfloat16)
    wl = rnd(c, k, scale=1 / 16, seed=14).to(torch.bfloat16)
    res = rnd(n * t, c, seed=15).to(torch.bfloat16)
    runs = []
    for _ in range(2):
        acc = acc_for(n)
        y = torch.empty(n * t, c, dtype=torch.bfloat16, device=dev)
        ops.linear(ctx, a, wl, n * t, c, y, resid=res, algo=algo or None, nsplit=nsplit or None,
                   gn=ops.gn_fuse_fwd([(acc, 0, G, c // G, t)]))
        runs.append((y, acc))
    torch.cuda.synchronize()
    y, acc = runs[0]
    # the block finishing a split tile (its last arriver) picks the replica, so compare the replica sums
    assert torch.equal(runs[1][0], y) and torch.equal(runs[1][1].view(4, -1).sum(0), acc.view(4, -1).sum(0))
    y0 = torch.empty_like(y)   # the fused epilogue stores what the plain one stores
    ops.linear(ctx, a, wl, n * t, c, y0, resid=res, algo=algo or None, nsplit=nsplit or None)
    torch.cuda.synchronize()
    assert torch.equal(y0, y)
    gamma = torch.ones(c, device=dev)
    beta = torch.zeros(c, device=dev)
    out = torch.empty_like(y)
    st = torch.empty(n, G, 2, device=dev)
    ops.groupnorm_acc(ctx, y, n, t, c, gamma, beta, 1e-6, False, acc, out, st)
    torch.cuda.synchronize()
    mean, var = group_stats(y, n, t, c)
    assert rel(st[..., 0], mean) < 1e-6 and rel(st[..., 1], (var + 1e-6).rsqrt()) < 1e-6


@pytest.mark.parametrize("silu,two,algo,nsplit", [(True, False, 3, 1), (True, True, 13, 2), (False, False, 1, -1),
                                                  (True, False, 31, 1), (True, True, 29, 2), (True, False, 62, 1),
                                                  (True, True, 63, 2), (False, False, 64, 1), (True, False, 43, 1),
                                                  (True, True, 44, -2), (False, False, 46, 2), (True, True, 47, -2)])
def test_fused_backward(ctx, silu, two, algo, nsplit):
    """Mode 2: the conv producing dL/d(GN(+SiLU) output) stores dy' and sums (gamma dy', gamma dy' xhat); the
    one-pass backward then matches torch autograd and the separate-pass kernels."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    n, h, w, c, cg = 2, 9, 12, 960, 128
    x = (rnd(n, c, h, w, seed=16) * 2 + 0.5).to(torch.bfloat16).float().requires_grad_(True)
    gamma = (1 + 0.1 * rnd(c, seed=17)).to(torch.bfloat16).float()
    beta = (0.1 * rnd(c, seed=18)).to(torch.bfloat16).float()
    xs = nhwc(x.detach())
    c1 = 640
    xa, xb = (xs[:, :c1].contiguous(), xs[:, c1:].contiguous()) if two else (xs, None)
    kx = dict(x2=xb, c1=c1) if two else {}
    y = torch.empty_like(xs)
    stats = torch.empty(n, G, 2, device=dev)
    ops.groupnorm(ctx, xa, n, h * w, c, gamma, beta, 1e-5, silu, y, stats, **kx)
    # the upstream gradient comes out of a conv (dgrad-like: cg -> c channels)
    gsrc = nhwc(rnd(n, cg, h, w, seed=19))
    wt = pack_conv(rnd(c, cg, 3, 3, scale=1 / math.sqrt(9 * cg), seed=20)).to(dev, torch.bfloat16)
    ckw = dict(nb=n, hin=h, win=w, cin=cg, hout=h, wout=w, cout=c, algo=algo, nsplit=nsplit)
    dy = torch.empty(n * h * w, c, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, gsrc, wt, y=dy, **ckw)
    acc = acc_for(n)
    dyp = torch.empty_like(dy)
    g = ops.gn_fuse_bwd(acc, G, c // G, h * w, xa, stats, gamma, beta, silu, **kx)
    ops.conv_gemm(ctx, gsrc, wt, y=dyp, gn=g, **ckw)
    add = nhwc(rnd(n, c, h, w, seed=21))
    dx = torch.empty_like(xs)
    ops.groupnorm_bwd_acc(ctx, xa, n, h * w, c, gamma, stats, acc, dyp, dx, add1=add, **kx)
    dx_sep = torch.empty_like(xs)
    ops.groupnorm_bwd(ctx, xa, n, h * w, c, gamma, beta, silu, stats, dy, dx_sep, add1=add, **kx)
    torch.cuda.synchronize()
    # dy' as autograd rounds it: dy * silu'(bf16(GN(x)))
    yv = F.group_norm(x.detach(), G, gamma, beta, eps=1e-5).to(torch.bfloat16).float()
    sg = torch.sigmoid(yv)
    dyp_ref = (nchw(dy, n, h, w) * (sg * (1 + yv * (1 - sg)))) if silu else nchw(dy, n, h, w)
    assert rel(nchw(dyp, n, h, w), dyp_ref) < 5e-3
    ref = F.group_norm(x, G, gamma, beta, eps=1e-5)
    if silu:
        ref = F.silu(ref)
    ref.backward(nchw(dy, n, h, w))
    assert rel(nchw(dx, n, h, w), x.grad + nchw(add, n, h, w)) < 2e-2
    assert rel(dx, dx_sep) < 5e-3


def test_fused_nonfinite_marks_nan(ctx):
    """A non-finite output value is counted: the statistics read back as NaN instead of a wrong finite value."""
    from depth_completion_amd import ops
    n, t, c, k = 1, 64, 64, 64
    a = rnd(n * t, k, seed=22).to(torch.bfloat16)
    a[5, 3] = float("inf")
    wl = rnd(c, k, seed=23).to(torch.bfloat16)
    acc = acc_for(n)
    y = torch.empty(n * t, c, dtype=torch.bfloat16, device=dev)
    ops.linear(ctx, a, wl, n * t, c, y, gn=ops.gn_fuse_fwd([(acc, 0, G, c // G, t)]))
    out = torch.empty_like(y)
    st = torch.empty(n, G, 2, device=dev)
    ops.groupnorm_acc(ctx, y, n, t, c, torch.ones(c, device=dev), torch.zeros(c, device=dev), 1e-6, False, acc, out,
                      st)
    torch.cuda.synchronize()
    assert bool(torch.isnan(st[0, :, 0]).any())


def test_fused_rejects_bad_targets(ctx):
    """Argument contract: a frame size that does not divide the rows, or a row list, is refused."""
    from depth_completion_amd import _lib, ops
    n, t, c, k = 1, 64, 64, 64
    a = rnd(n * t, k, seed=24).to(torch.bfloat16)
    wl = rnd(c, k, seed=25).to(torch.bfloat16)
    acc = acc_for(n)
    y = torch.empty(n * t, c, dtype=torch.bfloat16, device=dev)
    with pytest.raises(_lib.DCError):
        ops.linear(ctx, a, wl, n * t, c, y, gn=ops.gn_fuse_fwd([(acc, 0, G, c // G, 48)]))
    with pytest.raises(_lib.DCError):
        ops.linear(ctx, a, wl, n * t, c, y, gn=ops.gn_fuse_fwd([(acc, 8, G, c // G, t)]))   # coff + cout > C


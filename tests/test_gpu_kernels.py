"""Per-kernel parity of libdcamd.so against plain PyTorch fp32 references of the same op (GPU).

Inputs are rounded to bf16 first, references run in fp32 on the same rounded values; the bar is a
relative L2 error (bf16 storage of outputs ~ 4e-3) stated per test.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = torch.device("cuda:0")


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


def nhwc(x):  # NCHW fp32 -> [N*H*W, C] bf16
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c).to(torch.bfloat16).contiguous()


def nchw(t, n, h, w):
    return t.float().reshape(n, h, w, -1).permute(0, 3, 1, 2)


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).float().to(dev)


# ----------------------------------------------------------------------------- conv / gemm
@pytest.mark.parametrize("n,cin,cout,h,w,stride", [
    (1, 64, 64, 9, 11, 1), (2, 320, 320, 12, 16, 1), (1, 128, 192, 7, 5, 2), (2, 640, 1280, 6, 8, 1),
    (1, 1280, 1280, 3, 4, 1), (1, 64, 4, 8, 8, 1), (1, 64, 3, 16, 12, 1)])
def test_conv3x3(ctx, n, cin, cout, h, w, stride):
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    x = rnd(n, cin, h, w, seed=1)
    wt = rnd(cout, cin, 3, 3, scale=1 / math.sqrt(9 * cin), seed=2)
    b = rnd(cout, seed=3)
    ref = F.conv2d(x, wt, b, stride=stride, padding=1)
    ho, wo = ref.shape[-2:]
    ldy = max(8, -(-cout // 8) * 8)
    y = torch.zeros(n * ho * wo, ldy, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, nhwc(x), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=h, win=w, cin=cin, hout=ho, wout=wo,
                  cout=cout, stride=stride, bias=b, y=y)
    torch.cuda.synchronize()
    assert rel(nchw(y[:, :cout], n, ho, wo), ref) < 1e-2


def test_conv_epilogues_and_concat(ctx):
    """two-source input, per-step row bias, residual, relu, relu-backward mask."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    n, c1, c2, cout, h, w = 2, 128, 64, 128, 6, 7
    xa, xb = rnd(n, c1, h, w, seed=4), rnd(n, c2, h, w, seed=5)
    wt = rnd(cout, c1 + c2, 3, 3, scale=0.05, seed=6)
    b = rnd(cout, seed=7)
    table = rnd(5, cout, seed=8)
    res = rnd(n, cout, h, w, seed=9)
    mask = rnd(n, cout, h, w, seed=10)
    ctx.step.fill_(3)
    y = torch.empty(n * h * w, cout, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, nhwc(xa), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=h, win=w, cin=c1 + c2, hout=h,
                  wout=w, cout=cout, x2=nhwc(xb), c1=c1, bias=b, rowbias=table.to(torch.bfloat16), rowbias_ld=cout,
                  resid=nhwc(res), act=1, mask=nhwc(mask), y=y)
    torch.cuda.synchronize()
    ctx.step.zero_()
    ref = F.conv2d(torch.cat([xa, xb], 1), wt, b, padding=1) + table[3].view(1, -1, 1, 1) + res
    ref = torch.relu(ref) * (mask > 0)
    assert rel(nchw(y, n, h, w), ref) < 1e-2


def test_linear_many_rows(ctx):
    """A linear over more rows than sqrt(2^31) (the batch-8 level-0 token count): the gather's 32-bit pixel
    arithmetic bounds pixel indices, and only the mode-1 upsample products beyond that."""
    from depth_completion_amd import ops
    rows, k, m = 55296, 64, 64
    a = rnd(rows, k, seed=60).to(torch.bfloat16)
    wl = rnd(m, k, scale=1 / 8, seed=61).to(torch.bfloat16)
    out = torch.empty(rows, m, dtype=torch.bfloat16, device=dev)
    ops.linear(ctx, a, wl, rows, m, out)
    torch.cuda.synchronize()
    assert rel(out, a.float() @ wl.float().t()) < 1e-2


def test_conv_upsample_mode(ctx):
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    n, c, h, w = 1, 64, 5, 7
    for ho, wo in ((10, 14), (9, 13)):
        x = rnd(n, c, h, w, seed=11)
        wt = rnd(c, c, 3, 3, scale=0.05, seed=12)
        ref = F.conv2d(F.interpolate(x, size=(ho, wo), mode="nearest"), wt, padding=1)
        y = torch.empty(n * ho * wo, c, dtype=torch.bfloat16, device=dev)
        ops.conv_gemm(ctx, nhwc(x), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=h, win=w, cin=c, hout=ho,
                      wout=wo, cout=c, mode=1, y=y)
        torch.cuda.synchronize()
        assert rel(nchw(y, n, ho, wo), ref) < 1e-2


@pytest.mark.parametrize("mode,algo,nsplit", [(0, 3, 1), (0, 13, 2), (1, 12, 1), (0, 0, 0)])
def test_conv_row_list(ctx, mode, algo, nsplit):
    """dc_conv_desc.rows: only the listed output pixels are computed (bitwise the dense result at those rows
    for the same tile / split), every other row left untouched; residual and ReLU-mask epilogues included."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    n, c, h, w = 2, 64, 24, 20
    hin, win = (h // 2, w // 2) if mode == 1 else (h, w)
    x = nhwc(rnd(n, c, hin, win, seed=13))
    wt = pack_conv(rnd(c, c, 3, 3, scale=0.05, seed=14)).to(dev, torch.bfloat16)
    b = rnd(c, seed=15)
    res = nhwc(rnd(n, c, h, w, seed=16))
    msk = nhwc(rnd(n, c, h, w, seed=17))
    kw = dict(nb=n, hin=hin, win=win, cin=c, hout=h, wout=w, cout=c, mode=mode, bias=b, resid=res, mask=msk,
              algo=algo, nsplit=nsplit)
    dense = torch.zeros(n * h * w, c, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, x, wt, y=dense, **kw)
    g = torch.Generator().manual_seed(18)
    sel = torch.randperm(n * h * w, generator=g)[:300].sort().values
    rows = torch.zeros(4096, dtype=torch.int32)
    rows[:300] = sel.int()
    rows[300:] = int(sel[-1])            # padding repeats the last pixel, as the pipeline pads
    rows = rows.to(dev)
    sparse = torch.full((n * h * w, c), 7.0, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, x, wt, y=sparse, rows=(rows, 4096 if algo else 300), **kw)
    torch.cuda.synchronize()
    sel_d = sel.to(dev)
    if algo:
        assert torch.equal(sparse[sel_d], dense[sel_d])
    else:   # heuristic tile / split for 300 rows: same values up to fp32 summation order
        assert rel(sparse[sel_d], dense[sel_d]) < 1e-2
    keep = torch.ones(n * h * w, dtype=torch.bool, device=dev)
    keep[sel_d] = False
    assert bool((sparse[keep] == 7.0).all())


@pytest.mark.parametrize("h,w", [(8, 10), (7, 9)])
def test_conv_dgrad_modes(ctx, h, w):
    """input-gradients: stride-1 (flipped weights), stride-2 (mode 2), vs autograd."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv_dgrad
    n, cin, cout = 2, 64, 128
    for stride in (1, 2):
        x = rnd(n, cin, h, w, seed=13).requires_grad_(True)
        wt = rnd(cout, cin, 3, 3, scale=0.05, seed=14)
        y = F.conv2d(x, wt, stride=stride, padding=1)
        gy = rnd(*y.shape, seed=15)
        y.backward(gy)
        ho, wo = y.shape[-2:]
        dx = torch.empty(n * h * w, cin, dtype=torch.bfloat16, device=dev)
        ops.conv_gemm(ctx, nhwc(gy), pack_conv_dgrad(wt).to(dev, torch.bfloat16), nb=n, hin=ho, win=wo, cin=cout,
                      hout=h, wout=w, cout=cin, mode=0 if stride == 1 else 2, y=dx)
        torch.cuda.synchronize()
        assert rel(nchw(dx, n, h, w), x.grad) < 1e-2, stride


def test_small_cin_and_splitk_linear(ctx):
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    # small-C path (cin 8, K padded to 128)
    n, cin, cout, h, w = 2, 8, 320, 6, 8
    x = rnd(n, cin, h, w, seed=16)
    wt = rnd(cout, cin, 3, 3, scale=0.1, seed=17)
    y = torch.empty(n * h * w, cout, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, nhwc(x), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=h, win=w, cin=cin, hout=h, wout=w,
                  cout=cout, y=y)
    torch.cuda.synchronize()
    assert rel(nchw(y, n, h, w), F.conv2d(x, wt, padding=1)) < 1e-2
    # linear with deep K and few rows -> split-K path
    rows, k, m = 100, 5120, 1280
    a = rnd(rows, k, seed=18)
    wl = rnd(m, k, scale=1 / math.sqrt(k), seed=19)
    b = rnd(m, seed=20)
    res = rnd(rows, m, seed=21)
    out = torch.empty(rows, m, dtype=torch.bfloat16, device=dev)
    ops.linear(ctx, a.to(torch.bfloat16), wl.to(torch.bfloat16), rows, m, out, bias=b, resid=res.to(torch.bfloat16))
    torch.cuda.synchronize()
    assert rel(out, a @ wl.t() + b + res) < 1e-2


# ----------------------------------------------------------------------------- norms
@pytest.fixture(params=["group", "2pass", "3pass"])
def gn_path(request, monkeypatch):
    """GroupNorm launch form: a single launch, one block per (frame, group), wherever the slice fits the LDS
    (DC_GN_GROUP=-1; by default only small slices take it), stats + apply with the finalize folded into every
    apply block (DC_GN_GROUP=0), or stats / finalize / apply (DC_GN_GROUP=0, DC_GN_FUSED=0)."""
    monkeypatch.setenv("DC_GN_GROUP", "-1" if request.param == "group" else "0")   # -1: no size cap
    monkeypatch.setenv("DC_GN_FUSED", "0" if request.param == "3pass" else "1")
    return request.param


@pytest.mark.parametrize("c,silu,two", [(320, True, False), (640, False, False), (960, True, True), (64, True, False),
                                        (1280, True, False)])
def test_groupnorm_fwd_bwd(ctx, gn_path, c, silu, two):
    from depth_completion_amd import ops
    n, h, w = 2, 9, 12
    x = rnd(n, c, h, w, seed=22) * 2 + 0.5
    x = x.to(torch.bfloat16).float().requires_grad_(True)
    gamma = (1 + 0.1 * rnd(c, seed=23)).to(torch.bfloat16).float()
    beta = (0.1 * rnd(c, seed=24)).to(torch.bfloat16).float()
    ref = F.group_norm(x, 32, gamma, beta, eps=1e-5)
    if silu:
        ref = F.silu(ref)
    gy = rnd(*ref.shape, seed=25)
    ref.backward(gy)
    xs = nhwc(x.detach())
    y = torch.empty_like(xs)
    stats = torch.empty(n, 32, 2, device=dev)
    c1 = 640 if two else 0
    if two:
        xa, xb = xs[:, :c1].contiguous(), xs[:, c1:].contiguous()
        ops.groupnorm(ctx, xa, n, h * w, c, gamma, beta, 1e-5, silu, y, stats, x2=xb, c1=c1)
    else:
        ops.groupnorm(ctx, xs, n, h * w, c, gamma, beta, 1e-5, silu, y, stats)
    dx = torch.empty_like(xs)
    add = nhwc(gy)
    if two:
        ops.groupnorm_bwd(ctx, xa, n, h * w, c, gamma, beta, silu, stats, nhwc(gy), dx, x2=xb, c1=c1, add1=add)
    else:
        ops.groupnorm_bwd(ctx, xs, n, h * w, c, gamma, beta, silu, stats, nhwc(gy), dx, add1=add)
    torch.cuda.synchronize()
    assert rel(nchw(y, n, h, w), ref) < 1e-2
    assert rel(nchw(dx, n, h, w), x.grad + gy) < 2e-2


@pytest.mark.parametrize("n,h,w,c", [(1, 72, 96, 320), (3, 24, 32, 640), (8, 18, 24, 1280), (1, 1, 5, 64)])
def test_groupnorm_many_chunks(ctx, gn_path, n, h, w, c):
    """GroupNorm where the stats pass spans many blocks (every apply block folds the frame's chunk
    partials): statistics against torch fp32, and repeated calls bit-identical."""
    from depth_completion_amd import ops
    x = (rnd(n, c, h, w, seed=40) * 1.5 - 0.3).to(torch.bfloat16).float()
    gamma = (1 + 0.1 * rnd(c, seed=41)).to(torch.bfloat16).float()
    beta = (0.1 * rnd(c, seed=42)).to(torch.bfloat16).float()
    xs = nhwc(x)
    outs = []
    for _ in range(3):
        y = torch.empty_like(xs)
        stats = torch.empty(n, 32, 2, device=dev)
        ops.groupnorm(ctx, xs, n, h * w, c, gamma, beta, 1e-5, True, y, stats)
        dx = torch.empty_like(xs)
        ops.groupnorm_bwd(ctx, xs, n, h * w, c, gamma, beta, True, stats, y, dx)
        outs.append((y, stats, dx))
    torch.cuda.synchronize()
    xg = x.view(n, 32, -1)
    assert rel(stats[..., 0], xg.mean(-1)) < 1e-4
    assert rel(stats[..., 1], (xg.var(-1, unbiased=False) + 1e-5).rsqrt()) < 1e-4
    assert rel(nchw(y, n, h, w), F.silu(F.group_norm(x, 32, gamma, beta, eps=1e-5))) < 1e-2
    for y2, st2, dx2 in outs[1:]:
        assert torch.equal(y2, outs[0][0]) and torch.equal(st2, outs[0][1]) and torch.equal(dx2, outs[0][2])


@pytest.mark.parametrize("n,h,w,c,two", [(1, 72, 96, 320, False), (2, 36, 48, 960, True), (1, 9, 12, 2560, True)])
def test_groupnorm_paths_agree(ctx, monkeypatch, n, h, w, c, two):
    """The single-launch and 3-launch GroupNorm give the same statistics (fp64 folds of fp32 partials in
    different orders: rel 1e-5) and outputs within a bf16 ulp's worth of rounding flips."""
    from depth_completion_amd import ops
    x = (rnd(n, c, h, w, seed=43) * 1.5 + 0.2).to(torch.bfloat16)
    gamma = (1 + 0.1 * rnd(c, seed=44)).to(torch.bfloat16).float()
    beta = (0.1 * rnd(c, seed=45)).to(torch.bfloat16).float()
    xs = nhwc(x)
    c1 = c // 3 * 2 // 8 * 8 if two else 0
    xa, xb = (xs[:, :c1].contiguous(), xs[:, c1:].contiguous()) if two else (xs, None)
    gy = nhwc(rnd(n, c, h, w, seed=46).to(torch.bfloat16))
    res = {}
    for path in ("group", "2pass", "3pass"):
        monkeypatch.setenv("DC_GN_GROUP", "-1" if path == "group" else "0")
        monkeypatch.setenv("DC_GN_FUSED", "0" if path == "3pass" else "1")
        y = torch.empty_like(xs)
        stats = torch.empty(n, 32, 2, device=dev)
        dx = torch.empty_like(xs)
        kw = dict(x2=xb, c1=c1) if two else {}
        ops.groupnorm(ctx, xa, n, h * w, c, gamma, beta, 1e-6, True, y, stats, **kw)
        ops.groupnorm_bwd(ctx, xa, n, h * w, c, gamma, beta, True, stats, gy, dx, **kw)
        torch.cuda.synchronize()
        res[path] = (y.float(), stats.clone(), dx.float())
    (y1, s1, d1), (y2, s2, d2), (y3, s3, d3) = res["group"], res["3pass"], res["2pass"]
    assert rel(s1, s2) < 1e-5
    assert rel(y1, y2) < 2e-3
    assert rel(d1, d2) < 5e-3
    # finalize folded into the apply blocks vs the finalize launch: the same fp32 partials, fp64 folds in two
    # fixed orders
    assert rel(s3, s2) < 1e-6
    assert rel(y3, y2) < 2e-3
    assert rel(d3, d2) < 5e-3


@pytest.mark.parametrize("c", [64, 320, 1280])
def test_layernorm_fwd_bwd(ctx, c):
    from depth_completion_amd import ops
    rows = 333
    x = (rnd(rows, c, seed=26) * 3 + 1).to(torch.bfloat16).float().requires_grad_(True)
    gamma = (1 + 0.1 * rnd(c, seed=27)).to(torch.bfloat16).float()
    beta = (0.1 * rnd(c, seed=28)).to(torch.bfloat16).float()
    ref = F.layer_norm(x, (c,), gamma, beta, 1e-5)
    gy = rnd(rows, c, seed=29)
    ref.backward(gy)
    y = torch.empty(rows, c, dtype=torch.bfloat16, device=dev)
    st = torch.empty(rows, 2, device=dev)
    ops.layernorm(ctx, x.detach().to(torch.bfloat16), rows, c, gamma, beta, 1e-5, y, st)
    dx = torch.empty_like(y)
    ops.layernorm_bwd(ctx, x.detach().to(torch.bfloat16), rows, c, gamma, st, gy.to(torch.bfloat16), dx)
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-2
    assert rel(dx, x.grad) < 2e-2


@pytest.mark.parametrize("c,n,geglu", [(320, 960, 0), (640, 1920, 0), (1280, 3840, 0), (320, 2560, 1),
                                        (1280, 10240, 1)])
@pytest.mark.parametrize("algo,nsplit", [(13, 1), (12, 1), (3, 1), (37, 1), (18, 1), (13, 3), (12, -1), (11, 1), (14, 1)])
def test_linear_ln_fused(ctx, c, n, geglu, algo, nsplit):
    """LayerNorm folded into the consuming linear (dc_ln_fuse: the rows' (mean, rstd) given, the normalisation
    applied in the epilogue after split-K / stream-K sums) against torch: bf16(LayerNorm(x)) @ W^T + bias in fp32.
    Rows with a large common offset check that the mean is subtracted after the product, on the folded weight's
    own column sums."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import LnLinear
    rows = 333
    x = (rnd(rows, c, seed=70) * 2 + 3 * rnd(rows, 1, seed=71)).to(torch.bfloat16).float()
    x[5] += 40.0   # |mean| >> std on one row
    x = x.to(torch.bfloat16).float()
    gamma = (1 + 0.2 * rnd(c, seed=72)).to(torch.bfloat16).float()
    beta = (0.2 * rnd(c, seed=73)).to(torch.bfloat16).float()
    w = rnd(n, c, scale=1 / math.sqrt(c), seed=74)
    b = 0.1 * rnd(n, seed=75)
    lin = LnLinear(w.cpu(), b.cpu(), gamma.cpu(), beta.cpu(), 1e-5, dev)
    l = F.layer_norm(x, (c,), gamma, beta, 1e-5).to(torch.bfloat16).float()
    ref = l @ w.to(torch.bfloat16).float().t() + b.to(torch.bfloat16).float()
    st = torch.stack([x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-5)], 1).contiguous()
    y = torch.zeros(rows, n, dtype=torch.bfloat16, device=dev)
    y2 = torch.zeros(rows, n // 2, dtype=torch.bfloat16, device=dev) if geglu else None
    f = ops.ln_fuse(lin, st)
    ops.linear(ctx, x.to(torch.bfloat16), lin.wf, rows, n, y, geglu=geglu, y2=y2, ln=f, algo=algo, nsplit=nsplit)
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-2
    # per row, so that the |mean| >> std row (where rstd * (acc - mean * csum) cancels) is not diluted by the others
    per_row = ((y.float() - ref).norm(dim=1) / ref.norm(dim=1)).max()
    assert rel(y[5], ref[5]) < 1e-2 and per_row < 2e-2, float(per_row)
    if geglu:
        hh = ref.view(rows, n // 16, 2, 8)[:, :, 0].reshape(rows, n // 2)
        gt = ref.view(rows, n // 16, 2, 8)[:, :, 1].reshape(rows, n // 2)
        assert rel(y2, hh * F.gelu(gt)) < 2e-2
    # the input-gradient through the folded weight is gamma * dL/dLN(x); with the LayerNorm backward (gamma NULL)
    # it gives dL/dx
    if not geglu and algo == 13 and nsplit == 1:
        xr = x.clone().requires_grad_(True)
        out = F.layer_norm(xr, (c,), gamma, beta, 1e-5) @ w.to(torch.bfloat16).float().t()
        gy = rnd(rows, n, seed=76)
        out.backward(gy)
        dl = torch.empty(rows, c, dtype=torch.bfloat16, device=dev)
        ops.linear(ctx, gy.to(torch.bfloat16), lin.wd, rows, c, dl)
        dx = torch.empty(rows, c, dtype=torch.bfloat16, device=dev)
        ops.layernorm_bwd(ctx, x.to(torch.bfloat16), rows, c, None, st, dl, dx)
        torch.cuda.synchronize()
        assert rel(dx, xr.grad) < 2e-2


# (64, 1) / (128, 2): the tiny UNet widths, where most waves of the block own no channel chunk
@pytest.mark.parametrize("C,heads", [(64, 1), (128, 2), (320, 5), (640, 10), (1280, 20)])
def test_cross_bwd_ln3_fused(ctx, C, heads):
    """dc_crossattn_bwd_ln (norm3 backward computed in the cross-attention backward's launch) equals
    dc_layernorm_bwd (gamma folded) followed by dc_crossattn_bwd bit for bit, ragged row count included."""
    from depth_completion_amd import ops
    rows = 333
    g = torch.Generator().manual_seed(77)
    U = (torch.randn(heads, C, generator=g) / math.sqrt(C)).to(dev)
    D = (torch.randn(heads, C, generator=g) / math.sqrt(C)).to(dev)
    gamma2 = (1 + 0.1 * torch.randn(C, generator=g)).to(torch.bfloat16).float().to(dev)
    beta2 = (0.1 * torch.randn(C, generator=g)).to(torch.bfloat16).float().to(dev)
    c0 = (0.1 * torch.randn(C, generator=g)).to(dev)
    r1 = rnd(rows, C, scale=2, seed=78).to(torch.bfloat16)
    tabs = ops.crossattn_tables(ctx, U, D, heads, C)
    r2 = torch.empty(rows, C, dtype=torch.bfloat16, device=dev)
    sl2 = torch.empty(rows, 2, device=dev)
    pr = torch.empty(rows, heads, device=dev)
    sl3 = torch.zeros(rows, 2, device=dev)
    ops.crossattn_fwd(ctx, r1, rows, C, heads, 1e-5, gamma2, beta2, tabs, c0, r2, sl2, pr, ystats=sl3, yeps=1e-5)
    # norm3's statistics of the output rows (dc_crossattn_fwd ystats) against torch on the stored bf16 rows
    r2f = r2.float()
    torch.testing.assert_close(sl3[:, 0], r2f.mean(1), rtol=0, atol=1e-5)
    torch.testing.assert_close(sl3[:, 1], torch.rsqrt(r2f.var(1, unbiased=False) + 1e-5), rtol=1e-5, atol=0)
    r2b = torch.empty_like(r2)
    ops.crossattn_fwd(ctx, r1, rows, C, heads, 1e-5, gamma2, beta2, tabs, c0, r2b, sl2, pr)
    assert torch.equal(r2, r2b)   # the statistics pass changes no output
    dl3 = rnd(rows, C, seed=79).to(torch.bfloat16)
    dr3 = rnd(rows, C, seed=80).to(torch.bfloat16)
    dr2 = torch.empty(rows, C, dtype=torch.bfloat16, device=dev)
    ops.layernorm_bwd(ctx, r2, rows, C, None, sl3, dl3, dr2, add=dr3)
    dx_a = torch.empty(rows, C, dtype=torch.bfloat16, device=dev)
    ops.crossattn_bwd(ctx, r1, rows, C, heads, gamma2, tabs, sl2, pr, dr2, dx_a)
    dx_b = torch.zeros(rows, C, dtype=torch.bfloat16, device=dev)
    ops.crossattn_bwd_ln(ctx, r1, rows, C, heads, gamma2, tabs, sl2, pr, dl3, r2, sl3, dr3, dx_b)
    torch.cuda.synchronize()
    assert torch.equal(dx_a, dx_b)


# ----------------------------------------------------------------------------- attention
# the last shape launches >= 1024 blocks (no key split), the others the 2-way key-split kernels
@pytest.mark.parametrize("n,t,heads", [(1, 64, 1), (2, 300, 2), (1, 1000, 5), (1, 108, 20), (16, 1000, 8)])
@pytest.mark.parametrize("cfg", [None, "0", "1", "2", "3", "4"])
def test_attention_fwd_bwd(ctx, n, t, heads, cfg, monkeypatch):
    """Every (query waves, key splits) block configuration (DC_ATTN_CFG) against fp32 SDPA."""
    from depth_completion_amd import ops
    if cfg is not None:
        if n * t * heads > 200000:
            pytest.skip("forced configurations are covered on the smaller shapes")
        monkeypatch.setenv("DC_ATTN_CFG", cfg)
    C = heads * 64
    qkv = rnd(n, t, 3 * C, seed=30).to(torch.bfloat16).float().requires_grad_(True)
    q, k, v = qkv.split(C, -1)
    sh = lambda z: z.view(n, t, heads, 64).transpose(1, 2)  # noqa: E731
    o = F.scaled_dot_product_attention(sh(q), sh(k), sh(v)).transpose(1, 2).reshape(n, t, C)
    do = rnd(n, t, C, seed=31)
    o.backward(do)
    qkv_b = qkv.detach().to(torch.bfloat16).reshape(n * t, 3 * C).contiguous()
    ob = torch.empty(n * t, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(n, heads, t, device=dev)
    ops.attn_fwd(ctx, qkv_b, n, t, heads, ob, lse)
    dq = torch.empty_like(qkv_b)
    delta = torch.empty(2, n, heads, t, device=dev)
    ops.attn_bwd(ctx, qkv_b, ob, do.to(torch.bfloat16).reshape(n * t, C), lse, n, t, heads, delta, dq)
    torch.cuda.synchronize()
    assert rel(ob.view(n, t, C), o) < 1e-2
    s = torch.einsum("nhqd,nhkd->nhqk", sh(q).detach(), sh(k).detach()) / 8
    assert rel(lse, torch.logsumexp(s, -1)) < 1e-4
    assert rel(dq.view(n, t, 3 * C), qkv.grad) < 2e-2


@pytest.mark.parametrize("n,t,heads,peak", [(1, 64, 1, 1.0), (1, 65, 2, 1.0), (2, 300, 2, 1.0), (1, 1000, 5, 1.0),
                                            (1, 1000, 5, 6.0), (1, 6912, 5, 1.0), (1, 6912, 5, 4.0)])
def test_attention_fwd_peaked(ctx, n, t, heads, peak):
    """Forward on peaked and unit-scale scores (`peak` scales the queries: rows whose running max moves by more than
    the lazy-rescale slack mid-sweep): bit-identical on repeat and against fp32 SDPA / logsumexp."""
    from depth_completion_amd import ops
    C = heads * 64
    qkv = rnd(n, t, 3 * C, seed=41).to(torch.bfloat16).float()
    qkv[..., :C] *= peak
    qkv = qkv.to(torch.bfloat16).float()
    q, k, v = qkv.split(C, -1)
    sh = lambda z: z.view(n, t, heads, 64).transpose(1, 2)  # noqa: E731
    ref = F.scaled_dot_product_attention(sh(q), sh(k), sh(v)).transpose(1, 2).reshape(n, t, C)
    lse_ref = torch.logsumexp(torch.einsum("nhqd,nhkd->nhqk", sh(q), sh(k)) / 8, -1)
    qkv_b = qkv.to(torch.bfloat16).reshape(n * t, 3 * C).contiguous()
    outs = {}
    for mode in ("a", "b"):
        ob = torch.zeros(n * t, C, dtype=torch.bfloat16, device=dev)
        lse = torch.zeros(n, heads, t, device=dev)
        ops.attn_fwd(ctx, qkv_b, n, t, heads, ob, lse)
        torch.cuda.synchronize()
        outs[mode] = (ob, lse)
    assert torch.equal(outs["a"][0], outs["b"][0]) and torch.equal(outs["a"][1], outs["b"][1])
    assert rel(outs["a"][0].view(n, t, C), ref) < 1e-2
    assert rel(outs["a"][1], lse_ref) < 1e-4


@pytest.mark.parametrize("n,t,heads", [(1, 300, 2), (2, 1000, 3), (1, 6912, 5)])
def test_attention_bwd_stream_k(ctx, n, t, heads, monkeypatch):
    """Stream-K backward (equal ranges of the flattened (block, tile) space over 2 blocks per CU, partials
    summed by the last-arriving block in block order): equal to the plain grid up to fp32 summation
    order, repeated calls bit-identical, and against fp32 SDPA.  (1, 300, 2) splits every key-block over
    5 one-tile blocks; (1, 6912, 5) is the UNet level-0 shape the default policy sends to stream-K."""
    from depth_completion_amd import ops
    C = heads * 64
    qkv = rnd(n, t, 3 * C, seed=32).to(torch.bfloat16).float().requires_grad_(True)
    q, k, v = qkv.split(C, -1)
    sh = lambda z: z.view(n, t, heads, 64).transpose(1, 2)  # noqa: E731
    o = F.scaled_dot_product_attention(sh(q), sh(k), sh(v)).transpose(1, 2).reshape(n, t, C)
    do = rnd(n, t, C, seed=33)
    o.backward(do)
    qkv_b = qkv.detach().to(torch.bfloat16).reshape(n * t, 3 * C).contiguous()
    dob = do.to(torch.bfloat16).reshape(n * t, C)
    ob = torch.empty(n * t, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(n, heads, t, device=dev)
    ops.attn_fwd(ctx, qkv_b, n, t, heads, ob, lse)
    outs = {}
    for mode in ("0", "2", "2b"):
        monkeypatch.setenv("DC_ATTN_SK", mode[0])
        dq = torch.zeros_like(qkv_b)
        delta = torch.empty(2, n, heads, t, device=dev)
        ops.attn_bwd(ctx, qkv_b, ob, dob, lse, n, t, heads, delta, dq)
        torch.cuda.synchronize()
        outs[mode] = dq
    assert torch.equal(outs["2"], outs["2b"])
    assert rel(outs["2"], outs["0"]) < 5e-3
    assert rel(outs["2"].view(n, t, 3 * C)[..., C:], qkv.grad[..., C:]) < 2e-2
    assert rel(outs["2"].view(n, t, 3 * C), qkv.grad) < 2e-2


@pytest.mark.parametrize("C,heads", [(64, 1), (128, 2), (320, 5), (640, 10), (1280, 20)])
def test_cross_attention_fold(ctx, C, heads):
    """Folded 2-key cross-attention == LN2 + attn2 (2-token context) + residual; the three UNet widths
    (U and D staged together in LDS at 320 / 640, one after the other at 1280 x 20 heads)."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import fold_cross_attention
    rows, cross = 257, 1024
    g = torch.Generator().manual_seed(32)
    sd = {"to_q.weight": torch.randn(C, C, generator=g) / math.sqrt(C),
          "to_k.weight": torch.randn(C, cross, generator=g) / math.sqrt(cross),
          "to_v.weight": torch.randn(C, cross, generator=g) / math.sqrt(cross),
          "to_out.0.weight": torch.randn(C, C, generator=g) / math.sqrt(C),
          "to_out.0.bias": torch.randn(C, generator=g) * 0.1}
    ctxt = torch.randn(2, cross, generator=g)
    U, D, c0 = [t.to(dev) for t in fold_cross_attention(sd, "", ctxt, heads)]
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(torch.bfloat16).float().to(dev)
    beta = (0.1 * torch.randn(C, generator=g)).to(torch.bfloat16).float().to(dev)
    x = (torch.randn(rows, C, generator=g) * 2).to(torch.bfloat16).float().to(dev).requires_grad_(True)
    bf = lambda t: t.to(torch.bfloat16).float().to(dev)  # noqa: E731
    nrm = F.layer_norm(x, (C,), gamma, beta, 1e-5)
    q = nrm @ bf(sd["to_q.weight"]).t()
    k = bf(ctxt) @ bf(sd["to_k.weight"]).t()
    v = bf(ctxt) @ bf(sd["to_v.weight"]).t()
    sh = lambda z: z.view(-1, heads, 64).transpose(0, 1)  # noqa: E731
    att = torch.softmax(sh(q) @ sh(k).transpose(1, 2) / 8, -1) @ sh(v)
    out = att.transpose(0, 1).reshape(rows, C) @ bf(sd["to_out.0.weight"]).t() + bf(sd["to_out.0.bias"]) + x
    dy = rnd(rows, C, seed=33)
    out.backward(dy)
    y = torch.empty(rows, C, dtype=torch.bfloat16, device=dev)
    st = torch.empty(rows, 2, device=dev)
    pr = torch.empty(rows, heads, device=dev)
    xb = x.detach().to(torch.bfloat16)
    tabs = ops.crossattn_tables(ctx, U, D, heads, C)
    ops.crossattn_fwd(ctx, xb, rows, C, heads, 1e-5, gamma, beta, tabs, c0, y, st, pr)
    dx = torch.empty_like(y)
    ops.crossattn_bwd(ctx, xb, rows, C, heads, gamma, tabs, st, pr, dy.to(torch.bfloat16), dx)
    torch.cuda.synchronize()
    assert rel(y, out) < 1e-2
    assert rel(dx, x.grad) < 2e-2
    # against the fold itself in fp32 with the kernel's bf16 rounding points (LN output, the residual sums): the
    # MFMA form's hi / lo bf16 operands keep ~16 mantissa bits of U, D and the sigmoids (the reference's LN
    # statistics sum in another order, so a few bf16-rounded LN outputs land one ulp apart: probs to 2e-3)
    xf = xb.float()
    mu = xf.mean(1, keepdim=True)
    rs = torch.rsqrt(((xf - mu) ** 2).mean(1, keepdim=True) + 1e-5)
    n = ((xf - mu) * rs * gamma + beta).to(torch.bfloat16).float()
    p = torch.sigmoid(n @ U.t())
    yf = ((p @ D + c0).to(torch.bfloat16).float() + xf)
    torch.testing.assert_close(pr, p, rtol=0, atol=2e-3)
    assert (pr - p).abs().mean() < 2e-5
    torch.testing.assert_close(st[:, 0], mu[:, 0], rtol=0, atol=1e-5)
    assert (y.float() - yf).abs().max() <= 4 * (yf.abs().max() * 2 ** -8)   # within a few bf16 ulps
    assert rel(y, yf) < 2e-3


# ----------------------------------------------------------------------------- elementwise
def test_geglu_and_upsample_adjoint(ctx):
    from depth_completion_amd import ops
    rows, c = 123, 256
    f = rnd(rows, 2 * c, seed=34).requires_grad_(True)
    hh, gg = f.chunk(2, -1)
    y = hh * F.gelu(gg)
    dy = rnd(rows, c, seed=35)
    y.backward(dy)
    yb = torch.empty(rows, c, dtype=torch.bfloat16, device=dev)
    ops.geglu(ctx, f.detach().to(torch.bfloat16), rows, c, yb)
    df = torch.empty(rows, 2 * c, dtype=torch.bfloat16, device=dev)
    ops.geglu_bwd(ctx, f.detach().to(torch.bfloat16), rows, c, dy.to(torch.bfloat16), df)
    torch.cuda.synchronize()
    assert rel(yb, y) < 1e-2 and rel(df, f.grad) < 2e-2
    # nearest-upsample adjoint (x2 and a non-integer size)
    for (hl, wl), (hh_, wh) in (((5, 7), (10, 14)), ((7, 12), (14, 24)), ((4, 12), (7, 24))):
        x = rnd(2, 64, hl, wl, seed=36).requires_grad_(True)
        up = F.interpolate(x, size=(hh_, wh), mode="nearest")
        g = rnd(*up.shape, seed=37)
        up.backward(g)
        out = torch.empty(2 * hl * wl, 64, dtype=torch.bfloat16, device=dev)
        ops.upsample_adjoint(ctx, nhwc(g), 2, hh_, wh, 64, hl, wl, out)
        torch.cuda.synchronize()
        assert rel(nchw(out, 2, hl, wl), x.grad) < 1e-2


@pytest.mark.parametrize("algo", list(range(1, 23)) + list(range(37, 43)) + list(range(59, 62)))   # the im2col ids
# (23 .. 36: halo, 43 .. 58: skinny / resident, 59 ..: wide tiles)
@pytest.mark.parametrize("nsplit", [1, 3, -1, -2])
def test_conv_all_algos(ctx, algo, nsplit):
    """every tile / ring variant, split-K (nsplit > 1) and stream-K (nsplit < 0: 256 / 512 blocks over
    the tile x k-chunk iterations, tiles cut between blocks) on conv (incl. concat, stride 2, upsample)
    and linear."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    cases = [(2, 128, 64, 192, 9, 10, 1, 0), (1, 64, 0, 128, 12, 8, 2, 0), (1, 64, 0, 64, 5, 7, 1, 1),
             (1, 320, 0, 320, 1, 200, 1, 0)]
    for n, c1, c2, cout, h, w, stride, mode in cases:
        cin = c1 + c2
        xa = rnd(n, c1, h, w, seed=40)
        xb = rnd(n, c2, h, w, seed=41) if c2 else None
        k = 1 if (h == 1 and cin == 320) else 3
        wt = rnd(cout, cin, k, k, scale=1 / math.sqrt(cin * k * k), seed=42)
        xin = torch.cat([xa, xb], 1) if c2 else xa
        if mode == 1:
            ho, wo = 2 * h, 2 * w
            ref = F.conv2d(F.interpolate(xin, size=(ho, wo), mode="nearest"), wt, padding=1)
        else:
            ref = F.conv2d(xin, wt, stride=stride, padding=k // 2)
            ho, wo = ref.shape[-2:]
        y = torch.empty(n * ho * wo, cout, dtype=torch.bfloat16, device=dev)
        ops.conv_gemm(ctx, nhwc(xa), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=h, win=w, cin=cin, hout=ho,
                      wout=wo, cout=cout, kh=k, kw=k, stride=stride, pad=k // 2, mode=mode,
                      x2=nhwc(xb) if c2 else None, c1=c1 if c2 else 0, y=y, algo=algo, nsplit=nsplit)
        torch.cuda.synchronize()
        assert rel(nchw(y, n, ho, wo), ref) < 1e-2, (algo, nsplit, n, cin, cout, h, w, stride, mode)


HALO_ALGOS = list(range(23, 37)) + list(range(62, 67))   # dc_conv_gemm algo ids of the halo-tile direct 3x3 conv
# (conv_gemm.hip; 62 ..: the round-4 192-px deep-ring variants)


@pytest.mark.parametrize("algo", HALO_ALGOS)
@pytest.mark.parametrize("nsplit", [1, 2, 3])
def test_conv_halo_algos(ctx, algo, nsplit):
    """halo-tile direct 3x3 conv, every variant, input channels split over blocks (split-K): direct and
    nearest-upsample (mode 1) inputs, two-source concat, batch 2, frames not a multiple of the spatial tile,
    output channels not a multiple of BN, and the full epilogue (bias, per-step row bias, residual, ReLU,
    ReLU-backward mask) vs torch fp32 on the bf16 values; bitwise reproducible run to run."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    assert _lib_num_algos() == NUM_ALGOS
    cases = [  # n, c1, c2, cout, h, w, mode, epilogue
        (2, 128, 64, 96, 9, 35, 0, True), (1, 64, 0, 64, 18, 24, 1, False), (1, 320, 0, 320, 9, 12, 0, True),
        (1, 64, 0, 32, 13, 70, 0, False)]
    for n, c1, c2, cout, h, w, mode, epi in cases:
        cin = c1 + c2
        hin, win = (h // 2, w // 2) if mode == 1 else (h, w)
        xa = rnd(n, c1, hin, win, seed=70)
        xb = rnd(n, c2, hin, win, seed=71) if c2 else None
        wt = rnd(cout, cin, 3, 3, scale=1 / math.sqrt(cin * 9), seed=72)
        xin = torch.cat([xa, xb], 1) if c2 else xa
        if mode == 1:
            xin = F.interpolate(xin, size=(h, w), mode="nearest")
        ref = F.conv2d(xin, wt, padding=1)
        kw = {}
        if epi:
            b = rnd(cout, seed=73)
            table = rnd(4, cout, seed=74)
            res = rnd(n, cout, h, w, seed=75)
            mask = rnd(n, cout, h, w, seed=76)
            ctx.step.fill_(2)
            ref = torch.relu(ref + b.view(1, -1, 1, 1) + table[2].view(1, -1, 1, 1) + res) * (mask > 0)
            kw = dict(bias=b, rowbias=table.to(torch.bfloat16), rowbias_ld=cout, resid=nhwc(res), act=1, mask=nhwc(mask))
        outs = []
        for _ in range(2):
            y = torch.full((n * h * w, cout), 3.0, dtype=torch.bfloat16, device=dev)
            ops.conv_gemm(ctx, nhwc(xa), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=hin, win=win, cin=cin,
                          hout=h, wout=w, cout=cout, mode=mode, x2=nhwc(xb) if c2 else None, c1=c1 if c2 else 0,
                          y=y, algo=algo, nsplit=nsplit, **kw)
            torch.cuda.synchronize()
            outs.append(y)
        ctx.step.zero_()
        assert rel(nchw(outs[0], n, h, w), ref) < 1e-2, (algo, nsplit, n, cin, cout, h, w, mode)
        assert torch.equal(outs[0], outs[1]), (algo, nsplit, n, cin, cout, h, w, mode)


SKINNY_FIRST, SKINNY_LAST = 43, 54   # dc_conv_gemm algo ids of the weight-streaming skinny variants (conv_skinny.h)
SKINNY_ALGOS = list(range(SKINNY_FIRST, SKINNY_LAST + 1))
RESIDENT_FIRST, RESIDENT_LAST = 55, 58   # ... of the weight-resident persistent narrow convs (conv_skinny.h)
NUM_ALGOS = 66   # 1 .. 61 (round 3) and the round-4 halo variants 62 .. 66


@pytest.mark.parametrize("algo", list(range(RESIDENT_FIRST, RESIDENT_LAST + 1)))
@pytest.mark.parametrize("bpc", [0, 1, 2])
def test_conv_resident_algos(ctx, algo, bpc):
    """weight-resident persistent 3x3 conv (cin 64, cout <= 64; bpc: blocks per CU of the persistent grid, 0 = as
    many as fit): direct and nearest-upsample input, batch 2 with frames not a multiple of the tile, more tiles than
    blocks (each block walks several, alternating halo slots), cout 64 / 48, the full epilogue (bias, residual,
    ReLU, ReLU-backward mask) vs torch fp32 on the bf16 values; shapes outside the contract (cout 3, cin 128) run
    the im2col heuristic; bitwise reproducible run to run."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    cases = [  # n, cin, cout, h, w, mode, epilogue
        (1, 64, 64, 144, 192, 0, True), (2, 64, 48, 37, 70, 0, False), (1, 64, 64, 72, 96, 1, True),
        (1, 64, 3, 40, 40, 0, False), (1, 128, 64, 18, 24, 0, False)]
    for n, cin, cout, h, w, mode, epi in cases:
        hin, win = (h // 2, w // 2) if mode == 1 else (h, w)
        x = rnd(n, cin, hin, win, seed=100)
        wt = rnd(cout, cin, 3, 3, scale=1 / math.sqrt(cin * 9), seed=101)
        xin = F.interpolate(x, size=(h, w), mode="nearest") if mode == 1 else x
        ref = F.conv2d(xin, wt, padding=1)
        kw = {}
        if epi:
            b = rnd(cout, seed=102)
            res = rnd(n, cout, h, w, seed=103)
            mask = rnd(n, cout, h, w, seed=104)
            ref = torch.relu(ref + b.view(1, -1, 1, 1) + res) * (mask > 0)
            kw = dict(bias=b, resid=nhwc(res), act=1, mask=nhwc(mask))
        outs = []
        for _ in range(2):
            ldy = -(-cout // 8) * 8
            y = torch.full((n * h * w, ldy), 3.0, dtype=torch.bfloat16, device=dev)
            ops.conv_gemm(ctx, nhwc(x), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=hin, win=win, cin=cin,
                          hout=h, wout=w, cout=cout, mode=mode, y=y, algo=algo, nsplit=bpc, **kw)
            torch.cuda.synchronize()
            outs.append(y[:, :cout])
        assert rel(nchw(outs[0].contiguous(), n, h, w), ref) < 1e-2, (algo, bpc, n, cin, cout, h, w, mode)
        assert torch.equal(outs[0], outs[1]), (algo, bpc, n, cin, cout, h, w, mode)


@pytest.mark.parametrize("algo", SKINNY_ALGOS)
@pytest.mark.parametrize("nsplit", [1, 2, 3, -2, -5])
def test_conv_skinny_algos(ctx, algo, nsplit):
    """weight-streaming skinny conv / linear, every variant (3x3 halo tiles and 1x1 row tiles), input chunks split
    over blocks (nsplit > 0: summed by the last-arriving block; < 0: by the second, reduce kernel): 3x3 direct /
    nearest-upsample / two-source concat, batch 2 with frames not a multiple of the tile,
    output channels not a multiple of the block's 64 / 128, linears over rows not a multiple of the row tile, and
    the full epilogue (bias, per-step row bias, residual, ReLU, ReLU-backward mask) vs torch fp32 on the bf16 values;
    a variant given a shape outside its contract runs the im2col heuristic; bitwise reproducible run to run."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    cases = [  # n, c1, c2, cout, h, w, k, mode, epilogue
        (1, 256, 0, 192, 9, 12, 3, 0, True), (2, 128, 128, 96, 7, 13, 3, 0, False), (1, 128, 0, 320, 18, 24, 3, 1, True),
        (1, 512, 0, 200, 1, 300, 1, 0, True), (2, 256, 256, 128, 9, 12, 1, 0, False), (1, 128, 0, 64, 5, 7, 3, 0, False)]
    for n, c1, c2, cout, h, w, k, mode, epi in cases:
        cin = c1 + c2
        hin, win = (h // 2, w // 2) if mode == 1 else (h, w)
        xa = rnd(n, c1, hin, win, seed=90)
        xb = rnd(n, c2, hin, win, seed=91) if c2 else None
        wt = rnd(cout, cin, k, k, scale=1 / math.sqrt(cin * k * k), seed=92)
        xin = torch.cat([xa, xb], 1) if c2 else xa
        if mode == 1:
            xin = F.interpolate(xin, size=(h, w), mode="nearest")
        ref = F.conv2d(xin, wt, padding=k // 2)
        kw = {}
        if epi:
            b = rnd(cout, seed=93)
            table = rnd(4, cout, seed=94)
            res = rnd(n, cout, h, w, seed=95)
            mask = rnd(n, cout, h, w, seed=96)
            ctx.step.fill_(1)
            ref = torch.relu(ref + b.view(1, -1, 1, 1) + table[1].view(1, -1, 1, 1) + res) * (mask > 0)
            kw = dict(bias=b, rowbias=table.to(torch.bfloat16), rowbias_ld=cout, resid=nhwc(res), act=1, mask=nhwc(mask))
        outs = []
        for _ in range(2):
            y = torch.full((n * h * w, cout), 3.0, dtype=torch.bfloat16, device=dev)
            ops.conv_gemm(ctx, nhwc(xa), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=hin, win=win, cin=cin,
                          hout=h, wout=w, cout=cout, kh=k, kw=k, pad=k // 2, mode=mode, x2=nhwc(xb) if c2 else None,
                          c1=c1 if c2 else 0, y=y, algo=algo, nsplit=nsplit, **kw)
            torch.cuda.synchronize()
            outs.append(y)
        ctx.step.zero_()
        assert rel(nchw(outs[0], n, h, w), ref) < 1e-2, (algo, nsplit, n, cin, cout, h, w, k, mode)
        assert torch.equal(outs[0], outs[1]), (algo, nsplit, n, cin, cout, h, w, k, mode)


def test_conv_halo_outside_contract_falls_back(ctx):
    """a halo algo id on a shape outside the halo contract (stride 2, 1x1, cin % 64 != 0: e.g. carried there by
    the nearest-tuned-shape pick) runs the im2col kernel instead, with the same result."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    for n, cin, cout, h, w, k, stride in ((1, 128, 64, 12, 10, 3, 2), (2, 64, 96, 6, 8, 1, 1), (1, 8, 64, 9, 9, 3, 1)):
        x = rnd(n, cin, h, w, seed=80)
        wt = rnd(cout, cin, k, k, scale=1 / math.sqrt(cin * k * k), seed=81)
        ref = F.conv2d(x, wt, stride=stride, padding=k // 2)
        ho, wo = ref.shape[-2:]
        y = torch.empty(n * ho * wo, cout, dtype=torch.bfloat16, device=dev)
        ops.conv_gemm(ctx, nhwc(x), pack_conv(wt).to(dev, torch.bfloat16), nb=n, hin=h, win=w, cin=cin, hout=ho,
                      wout=wo, cout=cout, kh=k, kw=k, stride=stride, pad=k // 2, y=y, algo=HALO_ALGOS[0], nsplit=2)
        torch.cuda.synchronize()
        assert rel(nchw(y, n, ho, wo), ref) < 1e-2, (n, cin, cout, h, w, k, stride)


def _lib_num_algos():
    from depth_completion_amd import _lib
    return _lib.load().dc_conv_num_algos()


@pytest.mark.parametrize("algo,nsplit", [(10, -1), (12, -2), (3, -3), (16, -1)])
def test_conv_stream_k_unet_shape_deterministic(ctx, algo, nsplit):
    """stream-K on a UNet L2 shape (M = 432, 3x3, 1280 -> 1280, bias + in-place residual): matches the
    plain-tile launch within bf16 rounding and is bitwise reproducible run to run."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import pack_conv
    n, c, h, w = 1, 1280, 18, 24
    x = rnd(n, c, h, w, seed=50)
    wt = rnd(c, c, 3, 3, scale=1 / math.sqrt(c * 9), seed=51)
    bias = rnd(c, seed=52).contiguous()
    res = rnd(n, c, h, w, seed=53)
    ref = F.conv2d(x, wt, bias=bias, padding=1) + res
    wp = pack_conv(wt).to(dev, torch.bfloat16)
    outs = []
    for _ in range(2):
        y = nhwc(res)
        ops.conv_gemm(ctx, nhwc(x), wp, nb=n, hin=h, win=w, cin=c, hout=h, wout=w, cout=c, bias=bias, resid=y,
                      y=y, algo=algo, nsplit=nsplit)
        torch.cuda.synchronize()
        outs.append(y.clone())
    assert rel(nchw(outs[0], n, h, w), ref) < 1e-2
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("algo,nsplit", [(0, 0), (17, 1), (10, 3), (12, -1)])
def test_geglu_epilogues(ctx, algo, nsplit):
    """GEGLU fused into FF1's epilogue (geglu = 1: interleaved pre-activation + h * gelu(gate)) and into
    FF2's input-gradient epilogue (geglu = 2: (dh, dgate) interleaved), vs torch fp32 on bf16 values."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import geglu_interleave
    rows, c, inner = 300, 128, 256
    x = rnd(rows, c, seed=60)
    w1 = rnd(2 * inner, c, scale=1 / math.sqrt(c), seed=61)
    b1 = rnd(2 * inner, seed=62)
    perm = geglu_interleave(2 * inner)
    f8 = torch.empty(rows, 2 * inner, dtype=torch.bfloat16, device=dev)
    gg = torch.empty(rows, inner, dtype=torch.bfloat16, device=dev)
    ops.linear(ctx, x.to(torch.bfloat16), w1[perm].to(torch.bfloat16).contiguous(), rows, 2 * inner, f8,
               bias=b1[perm].contiguous(), geglu=1, y2=gg)
    torch.cuda.synchronize()
    pre = (x @ w1.t() + b1).to(torch.bfloat16).float()
    h, g = pre[:, :inner], pre[:, inner:]
    assert rel(f8.float(), pre[:, perm]) < 1e-2
    assert rel(gg.float(), h * F.gelu(g).to(torch.bfloat16).float()) < 1e-2
    # backward: dgg = dr @ W2 (W2 [c2][inner] as the FF2 weight, its dgrad weight is W2^T [inner][c2])
    c2 = 192
    dr = rnd(rows, c2, seed=63)
    w2 = rnd(c2, inner, scale=1 / math.sqrt(inner), seed=64)
    df = torch.empty(rows, 2 * inner, dtype=torch.bfloat16, device=dev)
    ops.linear(ctx, dr.to(torch.bfloat16), w2.t().contiguous().to(torch.bfloat16), rows, inner, df, geglu=2,
               aux=f8, algo=algo or None, nsplit=nsplit or None)
    torch.cuda.synchronize()
    dgg = (dr @ w2).to(torch.bfloat16).float()
    hh, gq = h.clone().requires_grad_(), g.clone().requires_grad_()
    (hh * F.gelu(gq)).backward(dgg)
    ref = torch.cat([hh.grad, gq.grad], 1)[:, perm]
    assert rel(df.float(), ref) < 1e-2


# (64, 300, 59, 1): a wide 320-column tile id, which would straddle geglu_n = 256 -- the library runs the 64 x 64 tile
@pytest.mark.parametrize("c,rows,algo,nsplit", [(256, 300, 0, 0), (256, 300, 13, 2), (256, 300, 12, -1),
                                                 (320, 6912, 0, 0), (64, 300, 59, 1)])
def test_folded_ff2_proj_out(ctx, c, rows, algo, nsplit):
    """FF2 + proj_out folded into one linear over [gg | r2] (weights.FoldedPair, dc_fold_linear_pair): the forward
    (two sources, K = 5C) against the two linears in fp32, and the input-gradient with the GEGLU backward on the first
    4C columns and plain dL/dr2 on the rest (dc_conv_desc.geglu_n) against the two input-gradient linears."""
    from depth_completion_amd import ops
    from depth_completion_amd.weights import FoldedPair
    k2 = 4 * c
    w2 = rnd(c, k2, scale=1 / math.sqrt(k2), seed=110).cpu()
    b2 = rnd(c, scale=0.1, seed=111).cpu()
    wp = rnd(c, c, scale=1 / math.sqrt(c), seed=112).cpu()
    bp = rnd(c, scale=0.1, seed=113).cpu()
    f = FoldedPair(w2, b2, wp, bp, dev)
    gg = rnd(rows, k2, seed=114).to(torch.bfloat16)
    r2 = rnd(rows, c, seed=115).to(torch.bfloat16)
    x = rnd(rows, c, seed=116).to(torch.bfloat16)
    out = torch.empty(rows, c, dtype=torch.bfloat16, device=dev)
    ops.conv_gemm(ctx, gg, f.wf, nb=1, hin=1, win=rows, cin=5 * c, hout=1, wout=rows, cout=c, kh=1, kw=1, pad=0,
                  x2=r2, c1=k2, bias=f.bias, resid=x, y=out, algo=algo or None, nsplit=nsplit or None)
    torch.cuda.synchronize()
    w2d, wpd = w2.to(dev).double(), wp.to(dev).double()
    ref = ((gg.double() @ w2d.t() + b2.to(dev).double() + r2.double()) @ wpd.t()) + bp.to(dev).double() + x.double()
    assert rel(out, ref) < 1e-2
    # input-gradient: df (GEGLU backward of dL/dgg) and dL/dr2 from one launch
    f8 = rnd(rows, 2 * k2, seed=117).to(torch.bfloat16)
    dout = rnd(rows, c, seed=118).to(torch.bfloat16)
    df = torch.empty(rows, 2 * k2, dtype=torch.bfloat16, device=dev)
    dr2 = torch.empty(rows, c, dtype=torch.bfloat16, device=dev)
    ops.linear(ctx, dout, f.wd, rows, 5 * c, df, geglu=2, aux=f8, y2=dr2, geglu_n=k2, algo=algo or None,
               nsplit=nsplit or None)
    df0 = torch.empty_like(df)
    dgg = (dout.double() @ wpd @ w2d).to(torch.bfloat16)   # the two linears' dL/dgg, rounded as the kernel rounds
    ops.linear(ctx, dgg.contiguous(), torch.eye(k2, device=dev, dtype=torch.bfloat16), rows, k2, df0, geglu=2, aux=f8)
    torch.cuda.synchronize()
    assert rel(dr2, dout.double() @ wpd) < 1e-2
    assert rel(df, df0) < 2e-2
    with pytest.raises(Exception):   # geglu_n without the GEGLU backward, or not a multiple of 256
        ops.linear(ctx, dout, f.wd, rows, 5 * c, df, y2=dr2, geglu_n=k2)
    with pytest.raises(Exception):
        ops.linear(ctx, dout, f.wd, rows, 5 * c, df, geglu=2, aux=f8, y2=dr2, geglu_n=k2 - 128)


@pytest.mark.parametrize("nbytes,offset", [(1 << 10, 0), (1769472, 0), (5 << 20, 4), (3 * (1 << 20) + 7, 3)])
def test_memset_in_graph_replays(nbytes, offset):
    """dc_memset_async captured in a hipGraph clears its whole range on every replay, after the buffer has been
    dirtied between replays (the guided step clears its dA map this way), and leaves the bytes around it."""
    from depth_completion_amd import _lib
    buf = torch.full((nbytes + 64,), 0xAB, dtype=torch.uint8, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _lib.call("dc_memset_async", buf.data_ptr() + offset, 0, nbytes, s.cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        _lib.call("dc_memset_async", buf.data_ptr() + offset, 0, nbytes, torch.cuda.current_stream().cuda_stream)
    for val in (0x11, 0xFF, 0x5A):
        buf.fill_(val)
        g.replay()
        torch.cuda.synchronize()
        b = buf.cpu()
        assert int(b[offset:offset + nbytes].count_nonzero()) == 0
        assert bool((b[:offset] == val).all()) and bool((b[offset + nbytes:] == val).all())

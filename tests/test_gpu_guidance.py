"""Guidance-loss kernels against torch autograd of the oracle's compute_affine_params / compute_loss
(oracle/pipeline_ref.py, restating marigold_dc.py:53-245) on a decoded map at the loss resolution
(identity resize, so dA is dL/dA pixel for pixel).

Bar: fp32 autograd reference; the kernels round the decode map and each gradient contribution to bf16
as the reference's bf16 autograd does, so the bound is a few bf16 ulps in norm (rel 2e-2).
"""
import pytest
import torch

from oracle.pipeline_ref import compute_affine_params, compute_loss

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")

FLAGS = {"l1": 1, "l2": 2, "edge": 4, "smooth": 8}


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _setup(n, H, W, npts, seed):
    g = torch.Generator().manual_seed(seed)
    out = torch.zeros(n * H * W, 8)
    out[:, :3] = torch.rand(n * H * W, 3, generator=g) * 0.8 + 0.1
    out = out.to(torch.bfloat16)
    img = (torch.rand(n, 3, H, W, generator=g) * 255).to(torch.uint8)
    idx = torch.zeros(n, H * W, dtype=torch.int32)
    gval = torch.zeros(n, H * W)
    masks = torch.zeros(n, 1, H, W)
    guides = torch.zeros(n, 1, H, W)
    for i in range(n):
        p = torch.randperm(H * W, generator=g)[:npts].sort().values
        v = torch.rand(npts, generator=g) * 0.9 + 0.05
        idx[i, :npts] = p.int()
        gval[i, :npts] = v
        masks.view(n, -1)[i, p] = 1.0
        guides.view(n, -1)[i, p] = v
    cnt = torch.full((n,), npts, dtype=torch.int32)
    params = torch.zeros(n, 8)
    params[:, 1] = 1.0
    params[:, 3] = 1.0
    params[:, 5] = 1.0
    params[:, 6] = npts
    # decode tail as decode_prediction forms it in bf16 (x*2-1, channel mean, clip, (x+1)/2)
    x = out[:, :3].float().view(n, H, W, 3)
    t = (x * 2).to(torch.bfloat16).float()
    t = (t - 1).to(torch.bfloat16).float()
    mean = (t.sum(-1) / 3).to(torch.bfloat16).float().clamp(-1, 1)
    A = ((mean + 1).to(torch.bfloat16).float() / 2).to(torch.bfloat16).float().view(n, 1, H, W)
    return out, img, idx, gval, cnt, params, masks, guides, A


@pytest.mark.parametrize("funcs", [["l1", "l2"], ["l1", "l2", "edge", "smooth"], ["l2", "smooth"]])
def test_closed_form_dense_loss_grad(funcs):
    from depth_completion_amd import _lib
    from depth_completion_amd.ops import Ctx
    ctx = Ctx(dev)
    n, H, W, npts = 2, 24, 32, 90
    out, img, idx, gval, cnt, params, masks, guides, A = _setup(n, H, W, npts, 5)
    # torch fp32 reference: s, sh = compute_affine_params(A) differentiated, d = clamp(s A + sh)
    a = A.clone().requires_grad_(True)
    s, sh = compute_affine_params(a, guides, masks)
    d = (s.view(n, 1, 1, 1) * a + sh.view(n, 1, 1, 1)).clamp(0.0, 1.0)
    loss = compute_loss(d, guides, masks, funcs, images=img.float())
    loss.sum().backward()
    ref = a.grad.view(n, H * W)
    out_d, img_d, idx_d, gval_d, cnt_d, par_d = (t.to(dev) for t in (out, img, idx, gval, cnt, params))
    gmap = torch.empty(n, H * W, device=dev)
    _lib.call("dc_guide_map", idx_d.data_ptr(), gval_d.data_ptr(), cnt_d.data_ptr(), n, H, W, gmap.data_ptr(),
              ctx.stream)
    st8 = torch.zeros(n, 8, device=dev)
    grad2 = torch.zeros(n, 2, device=dev)
    dA = torch.zeros(n, H * W, device=dev)
    lossv = torch.zeros(n, device=dev)
    ws = torch.empty(-(-_lib.load().dc_dense_loss_ws_bytes(n, H, W) // 4), device=dev)
    geo = (8, n, H, W, H, W, H, W)
    _lib.call("dc_closed_form_stats", out_d.data_ptr(), *geo, idx_d.data_ptr(), gval_d.data_ptr(), cnt_d.data_ptr(),
              par_d.data_ptr(), st8.data_ptr(), ctx.stream)
    flags = sum(FLAGS[f] for f in funcs)
    _lib.call("dc_dense_loss", out_d.data_ptr(), *geo, img_d.data_ptr(), gmap.data_ptr(), cnt_d.data_ptr(),
              par_d.data_ptr(), st8.data_ptr(), flags | 16, ws.data_ptr(), dA.data_ptr(), grad2.data_ptr(),
              lossv.data_ptr(), ctx.stream)
    _lib.call("dc_closed_form_adjoint", out_d.data_ptr(), *geo, idx_d.data_ptr(), gval_d.data_ptr(),
              cnt_d.data_ptr(), par_d.data_ptr(), st8.data_ptr(), grad2.data_ptr(), dA.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    print(f"\ncf {funcs}: loss {lossv.tolist()} vs {loss.tolist()}; dA rel {rel(dA.cpu(), ref):.2e}; "
          f"scale {st8[:, 0].tolist()} vs {s.tolist()}")
    assert torch.allclose(st8[:, 0].cpu(), s.detach(), rtol=1e-2)
    assert torch.allclose(lossv.cpu(), loss.detach(), rtol=1e-3, atol=1e-5)
    assert rel(dA.cpu(), ref) < 2e-2
    if funcs == ["l1", "l2"]:   # the sparse-only kernel gives the same gradient
        dA2 = torch.zeros_like(dA)
        l2 = torch.zeros_like(lossv)
        _lib.call("dc_sparse_loss_cf", out_d.data_ptr(), *geo, idx_d.data_ptr(), gval_d.data_ptr(),
                  cnt_d.data_ptr(), par_d.data_ptr(), dA2.data_ptr(), l2.data_ptr(), ctx.stream)
        torch.cuda.synchronize()
        assert rel(dA, dA2) < 1e-2


@pytest.mark.parametrize("funcs", [["l1", "l2", "smooth"], ["l1", "edge"]])
def test_per_input_dense_loss_grad(funcs):
    """flags 32 | 64: unclamped learned-affine map, affine gradient only (per-input training)."""
    from depth_completion_amd import _lib
    from depth_completion_amd.ops import Ctx
    ctx = Ctx(dev)
    n, H, W, npts = 2, 24, 32, 90
    out, img, idx, gval, cnt, params, masks, guides, A = _setup(n, H, W, npts, 6)
    aff = torch.tensor([[1.1, 0.3], [0.9, 0.2]])
    sc = aff[:, 0].clone().requires_grad_(True)
    sh = aff[:, 1].clone().requires_grad_(True)
    d = (sc ** 2).view(n, 1, 1, 1) * A + (sh ** 2).view(n, 1, 1, 1) * 0.0   # min_g = 0, max_g = 1
    loss = compute_loss(d, guides, masks, funcs, images=img.float())
    loss.sum().backward()
    out_d, img_d, idx_d, gval_d, cnt_d, par_d = (t.to(dev) for t in (out, img, idx, gval, cnt, params))
    gmap = torch.empty(n, H * W, device=dev)
    _lib.call("dc_guide_map", idx_d.data_ptr(), gval_d.data_ptr(), cnt_d.data_ptr(), n, H, W, gmap.data_ptr(),
              ctx.stream)
    grad2 = torch.zeros(n, 2, device=dev)
    lossv = torch.zeros(n, device=dev)
    ws = torch.empty(-(-_lib.load().dc_dense_loss_ws_bytes(n, H, W) // 4), device=dev)
    aff_d = aff.to(dev)
    flags = sum(FLAGS[f] for f in funcs)
    _lib.call("dc_dense_loss", out_d.data_ptr(), 8, n, H, W, H, W, H, W, img_d.data_ptr(), gmap.data_ptr(),
              cnt_d.data_ptr(), par_d.data_ptr(), aff_d.data_ptr(), flags | 32 | 64, ws.data_ptr(), None,
              grad2.data_ptr(), lossv.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    assert torch.allclose(lossv.cpu(), loss.detach(), rtol=1e-3, atol=1e-5)
    assert torch.allclose(grad2[:, 0].cpu(), sc.grad, rtol=2e-3, atol=1e-5)


@pytest.mark.parametrize("ph,pw,rh,rw,h,w,nearest", [(48, 64, 48, 64, 48, 64, 0), (48, 64, 45, 60, 90, 120, 0),
                                                    (48, 64, 45, 60, 90, 120, 1), (16, 24, 16, 24, 37, 50, 0)])
def test_decode_row_sets(ph, pw, rh, rw, h, w, nearest):
    """dc_tap_mask / dc_dilate_mask / dc_mask_count + dc_mask_rows against a torch restatement: the resize taps
    of the sparse pixels (upsample_bilinear2d align_corners=False source indices, or nearest), 3x3 dilation
    within each frame, sorted compaction with the pad repeating the last index."""
    import torch.nn.functional as F
    from depth_completion_amd import _lib
    from depth_completion_amd.ops import Ctx
    ctx = Ctx(dev)
    n, npts = 2, 70
    g = torch.Generator().manual_seed(7)
    idx = torch.zeros(n, h * w, dtype=torch.int32)
    ref = torch.zeros(n, ph, pw, dtype=torch.bool)
    for i in range(n):
        p = torch.randperm(h * w, generator=g)[:npts].sort().values
        idx[i, :npts] = p.int()
        for q in p.tolist():
            y, x = divmod(q, w)
            if nearest:
                ys = [y if rh == h else min(int(y * (rh / h)), rh - 1)]
                xs = [x if rw == w else min(int(x * (rw / w)), rw - 1)]
            elif rh == h and rw == w:
                ys, xs = [y], [x]
            else:
                sy = max((rh / h) * (y + 0.5) - 0.5, 0.0)
                sx = max((rw / w) * (x + 0.5) - 0.5, 0.0)
                y0, x0 = int(sy), int(sx)
                ys = [y0, y0 + (1 if y0 < rh - 1 else 0)]
                xs = [x0, x0 + (1 if x0 < rw - 1 else 0)]
            for yy in ys:
                for xx in xs:
                    ref[i, yy, xx] = True
    params = torch.zeros(n, 8)
    params[:, 7] = 8.0 * nearest
    cnt = torch.full((n,), npts, dtype=torch.int32)
    idx_d, cnt_d, par_d = idx.to(dev), cnt.to(dev), params.to(dev)
    total = n * ph * pw
    m0 = torch.empty(total, dtype=torch.uint8, device=dev)
    m1 = torch.empty(total, dtype=torch.uint8, device=dev)
    _lib.call("dc_tap_mask", idx_d.data_ptr(), cnt_d.data_ptr(), par_d.data_ptr(), n, ph, pw, rh, rw, h, w,
              m0.data_ptr(), ctx.stream)
    _lib.call("dc_dilate_mask", m0.data_ptr(), n, ph, pw, m1.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    assert torch.equal(m0.view(n, ph, pw).bool().cpu(), ref)
    dil = F.max_pool2d(ref.float()[:, None], 3, stride=1, padding=1)[:, 0] > 0
    assert torch.equal(m1.view(n, ph, pw).bool().cpu(), dil)
    ws = torch.empty(-(-_lib.load().dc_mask_rows_ws_bytes(total) // 4), dtype=torch.int32, device=dev)
    cntr = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("dc_mask_count", m1.data_ptr(), total, ws.data_ptr(), cntr.data_ptr(), ctx.stream)
    c = int(cntr.item())
    want = torch.nonzero(dil.flatten()).flatten().int()
    assert c == want.numel()
    pad = c + 37
    rows = torch.full((pad,), -1, dtype=torch.int32, device=dev)
    _lib.call("dc_mask_rows", m1.data_ptr(), total, ws.data_ptr(), cntr.data_ptr(), pad, rows.data_ptr(),
              ctx.stream)
    torch.cuda.synchronize()
    rows = rows.cpu()
    assert torch.equal(rows[:c], want)
    assert bool((rows[c:] == want[-1]).all())

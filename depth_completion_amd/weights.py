"""Weight packing: diffusers-format state dicts -> device layouts of the HIP kernels.

* conv  [cout][cin][kh][kw]  -> forward  [cout][ktot]  K order (ky, kx, cin), cin padded to 8,
                                ktot padded to 64 (dc_conv_desc contract)
                             -> input-gradient W'[cin][ky][kx][cout] = W[cout][cin][kh-1-ky][kw-1-kx]
* linear [out][in]           -> forward as-is, input-gradient = W^T
* the folded 2-key cross-attention constants U, D, c0 (DESIGN.md "cross-attention")
This is a one-time, load-time layout transform (like a checkpoint converter); nothing here runs per step.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16


def _pad_k(t: torch.Tensor) -> torch.Tensor:
    k = t.shape[1]
    kt = -(-k // 64) * 64
    return F.pad(t, (0, kt - k)) if kt != k else t


def pack_conv(w: torch.Tensor, cin_pad: int | None = None) -> torch.Tensor:
    co, ci, kh, kw = w.shape
    cp = cin_pad or ci
    t = torch.zeros(co, kh, kw, cp, dtype=torch.float32)
    t[..., :ci] = w.float().permute(0, 2, 3, 1)
    return _pad_k(t.reshape(co, -1)).contiguous()


def pack_conv_dgrad(w: torch.Tensor, rows=None, cout_pad: int | None = None) -> torch.Tensor:
    wd = w.float().flip(2, 3).permute(1, 0, 2, 3)  # [cin][cout][kh][kw]
    if rows is not None:
        wd = wd[rows]
    return pack_conv(wd, cin_pad=cout_pad)


def round_bf16(t: torch.Tensor) -> torch.Tensor:
    return t.to(BF16).float()


class Conv:
    """A conv with forward and input-gradient packings on the device."""

    def __init__(self, w, b, device, *, stride=1, cin_pad=None, dgrad=True, dgrad_rows=None, dgrad_cout_pad=None):
        w = round_bf16(w)  # the reference runs bf16 weights (predict.py:474-488, torch_dtype=bf16)
        self.cout, self.cin, self.kh, self.kw = w.shape
        self.stride = stride
        self.pad = self.kh // 2
        self.cin_p = cin_pad or self.cin
        self.wf = pack_conv(w, cin_pad).to(device=device, dtype=BF16)
        self.bias = b.float().to(BF16).float().to(device) if b is not None else None
        self.wd = None
        if dgrad:
            self.dg_cout = len(dgrad_rows) if dgrad_rows is not None else self.cin
            self.dg_cin_p = dgrad_cout_pad or self.cout
            self.wd = pack_conv_dgrad(w, dgrad_rows, dgrad_cout_pad).to(device=device, dtype=BF16)


class Linear:
    def __init__(self, w, b, device, dgrad=True):
        w = round_bf16(w)
        self.cout, self.cin = w.shape
        self.wf = w.contiguous().to(device=device, dtype=BF16)
        self.bias = b.float().to(BF16).float().to(device) if b is not None else None
        self.wd = w.t().contiguous().to(device=device, dtype=BF16) if dgrad else None


class LnLinear:
    """A linear whose input is LayerNorm(x) (BasicTransformerBlock norm3 -> ff.net.0.proj), with the LayerNorm folded
    in (include/dcamd.h dc_ln_fuse): wf = bf16(W diag(gamma)) and its input-gradient wd = wf^T (which yields
    gamma * dL/dLN(x) for the LayerNorm backward), csum[n] = sum_k wf[n][k], cbias[n] = W[n] . beta + bias[n].
    Computed by the library's dc_fold_layernorm (host code shared with the native session)."""

    def __init__(self, w, b, norm_w, norm_b, eps, device):
        from . import _lib

        w = round_bf16(w).contiguous()
        self.cout, self.cin = w.shape
        self.eps = eps
        g = round_bf16(norm_w).contiguous()
        be = round_bf16(norm_b).contiguous()
        bias = b.float().to(BF16).float().contiguous() if b is not None else None
        wf = torch.empty(self.cout, self.cin, dtype=BF16)
        csum = torch.empty(self.cout, dtype=torch.float32)
        cbias = torch.empty(self.cout, dtype=torch.float32)
        _lib.call("dc_fold_layernorm", w.data_ptr(), self.cout, self.cin, g.data_ptr(), be.data_ptr(),
                  bias.data_ptr() if bias is not None else None, wf.data_ptr(), csum.data_ptr(), cbias.data_ptr())
        self.wf = wf.to(device)
        self.wd = wf.t().contiguous().to(device)
        self.csum = csum.to(device)
        self.cbias = cbias.to(device)


def geglu_interleave(n_out: int) -> torch.Tensor:
    """Row order of the GEGLU projection (ff.net.0.proj, [2 * inner][C]) for the fused epilogue of
    dc_conv_gemm (geglu = 1 / 2): blocks of 8 h rows then the 8 matching gate rows."""
    inner = n_out // 2
    blk = torch.arange(0, inner, 8)
    idx = torch.stack([blk[:, None] + torch.arange(8), inner + blk[:, None] + torch.arange(8)], 1)
    return idx.reshape(-1)


class Norm:
    def __init__(self, w, b, device, eps):
        self.gamma = round_bf16(w).to(device)
        self.beta = round_bf16(b).to(device)
        self.eps = eps


class FoldedPair:
    """FF2 (ff.net.2) and proj_out of a transformer block folded into one two-source linear over [gg | r2]
    (include/dcamd.h dc_fold_linear_pair): out = gg (Wp W2)^T + r2 Wp^T + (Wp b2 + bp) + x, with wf = [bf16(Wp W2) |
    Wp] [C][5C] and its input-gradient wd = wf^T [5C][C] (columns < 4C: dL/dgg for the GEGLU backward, the rest
    dL/dr2).  Computed by the library's host function (shared with the native session)."""

    def __init__(self, w2, b2, wp, bp, device):
        from . import _lib

        w2 = round_bf16(w2).contiguous()
        wp = round_bf16(wp).contiguous()
        c, k2 = w2.shape
        b2 = b2.float().to(BF16).float().contiguous()
        bp = bp.float().to(BF16).float().contiguous()
        wf = torch.empty(c, k2 + c, dtype=BF16)
        wd = torch.empty(k2 + c, c, dtype=BF16)
        bias = torch.empty(c, dtype=torch.float32)
        _lib.call("dc_fold_linear_pair", w2.data_ptr(), b2.data_ptr(), c, k2, wp.data_ptr(), bp.data_ptr(),
                  wf.data_ptr(), wd.data_ptr(), bias.data_ptr())
        self.cout, self.k2 = c, k2
        self.wf = wf.to(device)
        self.wd = wd.to(device)
        self.bias = bias.to(device)


def fold_cross_attention(sd: dict, pre: str, ctx: torch.Tensor, heads: int):
    """attn2 with a constant 2-token context -> (U [H][C], D [H][C], c0 [C]) in fp32.

    softmax over 2 keys: p0 = sigmoid(q.(k0-k1)/sqrt(64)); out = v1 + p0 (v0 - v1) per head, so
    attn2(n) = Wo(v1) + bo + sum_h p0_h Wo_h(v0_h - v1_h),  p0_h = sigmoid(n . U_h),
    U_h = Wq_h^T (k0_h - k1_h) / 8,  D_h = Wo_h (v0_h - v1_h),  c0 = Wo v1 + bo,
    in double from the bf16-rounded weights, k and v rounded to bf16 as the reference computes them (to_k / to_v
    in bf16).  Computed by the library's dc_fold_cross_attention (host code shared with the native session).
    """
    from . import _lib

    def f32(t):
        return t.detach().float().contiguous().cpu()
    wq, wk, wv = f32(sd[pre + "to_q.weight"]), f32(sd[pre + "to_k.weight"]), f32(sd[pre + "to_v.weight"])
    wo, bo = f32(sd[pre + "to_out.0.weight"]), f32(sd[pre + "to_out.0.bias"])
    c = f32(ctx.reshape(-1, ctx.shape[-1]))
    inner, C = wq.shape
    cout = wo.shape[0]
    U = torch.empty(heads, C, dtype=torch.float32)
    D = torch.empty(heads, cout, dtype=torch.float32)
    c0 = torch.empty(cout, dtype=torch.float32)
    _lib.call("dc_fold_cross_attention", wq.data_ptr(), wk.data_ptr(), wv.data_ptr(), wo.data_ptr(), bo.data_ptr(),
              c.data_ptr(), c.shape[0], inner, C, wk.shape[1], cout, heads, U.data_ptr(), D.data_ptr(), c0.data_ptr())
    return U, D, c0

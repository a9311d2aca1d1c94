"""AutoencoderKL (the Stable Diffusion VAE of ``--vae original``, predict.py:44-52) on HIP kernels.

Encoder forward replaces ``prepare_latents`` -> ``vae.encode(x).latent_dist.mode() * scaling_factor``
(marigold_dc.py:696-698); decoder forward + input-gradient replace ``decode_prediction`` ->
``vae.decode(z / scaling_factor)`` inside ``_latent_to_affine`` (marigold_dc.py:366) and its part of
``losses.backward`` (:877).  Module structure as diffusers 0.31.0 (restated in oracle/vae_kl_ref.py):
ResnetBlock2D without time embedding (GroupNorm 32, eps 1e-6, SiLU), DownEncoderBlock2D /
UpDecoderBlock2D, the mid block's single-head attention (head dim = channels), Downsample2D with the
(0, 1, 0, 1) pad, nearest Upsample2D + conv.  Convs / linears run on dc_conv_gemm, norms on
dc_groupnorm_*, the attention as GEMMs around dc_softmax_rows (csrc/vae_kl.hip).  The latent scale of
the encoder output is folded into quant_conv's mean rows.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from . import _lib, ops
from .ops import BF16, Ctx
from .weights import Conv, Linear, Norm


@dataclass
class KLConfig:
    block_out_channels: tuple = (128, 256, 512, 512)
    layers_per_block: int = 2
    latent_channels: int = 4
    scaling_factor: float = 0.18215


SD_VAE = KLConfig()
TINY_KL = KLConfig(block_out_channels=(32, 32, 64, 64), layers_per_block=1)


class _Res:
    def __init__(self, sd, pre, dev, cin, cout, dgrad):
        self.cin, self.cout = cin, cout
        self.norm1 = Norm(sd[pre + "norm1.weight"], sd[pre + "norm1.bias"], dev, 1e-6)
        self.conv1 = Conv(sd[pre + "conv1.weight"], sd[pre + "conv1.bias"], dev, dgrad=dgrad)
        self.norm2 = Norm(sd[pre + "norm2.weight"], sd[pre + "norm2.bias"], dev, 1e-6)
        self.conv2 = Conv(sd[pre + "conv2.weight"], sd[pre + "conv2.bias"], dev, dgrad=dgrad)
        self.shortcut = None
        if cin != cout:
            self.shortcut = Conv(sd[pre + "conv_shortcut.weight"], sd[pre + "conv_shortcut.bias"], dev, dgrad=dgrad)


class _Attn:
    def __init__(self, sd, pre, dev, c, dgrad):
        self.c = c
        self.norm = Norm(sd[pre + "group_norm.weight"], sd[pre + "group_norm.bias"], dev, 1e-6)
        self.q = Linear(sd[pre + "to_q.weight"], sd[pre + "to_q.bias"], dev, dgrad=dgrad)
        self.k = Linear(sd[pre + "to_k.weight"], sd[pre + "to_k.bias"], dev, dgrad=dgrad)
        self.v = Linear(sd[pre + "to_v.weight"], sd[pre + "to_v.bias"], dev, dgrad=dgrad)
        self.o = Linear(sd[pre + "to_out.0.weight"], sd[pre + "to_out.0.bias"], dev, dgrad=dgrad)


class AutoencoderKLHIP:
    def __init__(self, sd: dict, device, cfg: KLConfig = SD_VAE):
        dev = torch.device(device)
        self.device, self.cfg = dev, cfg
        ch = cfg.block_out_channels
        lc = cfg.latent_channels
        L = cfg.layers_per_block
        # ---- encoder (forward only)
        self.enc_in = Conv(sd["encoder.conv_in.weight"], sd["encoder.conv_in.bias"], dev, cin_pad=8, dgrad=False)
        self.enc_blocks = []
        prev = ch[0]
        for i, c in enumerate(ch):
            res = [_Res(sd, f"encoder.down_blocks.{i}.resnets.{j}.", dev, prev if j == 0 else c, c, False)
                   for j in range(L)]
            down = None
            if i < len(ch) - 1:
                down = Conv(sd[f"encoder.down_blocks.{i}.downsamplers.0.conv.weight"],
                            sd[f"encoder.down_blocks.{i}.downsamplers.0.conv.bias"], dev, stride=2, dgrad=False)
            self.enc_blocks.append((res, down))
            prev = c
        self.enc_mid = self._mid(sd, "encoder.mid_block.", dev, ch[-1], False)
        self.enc_norm = Norm(sd["encoder.conv_norm_out.weight"], sd["encoder.conv_norm_out.bias"], dev, 1e-6)
        self.enc_out = Conv(sd["encoder.conv_out.weight"], sd["encoder.conv_out.bias"], dev, dgrad=False)
        # quant_conv rows 0..lc-1 (the posterior mean = mode()), times scaling_factor
        s = cfg.scaling_factor
        qw = sd["quant_conv.weight"][:lc].float() * s
        qb = sd["quant_conv.bias"][:lc].float() * s
        self.quant = Conv(qw, qb, dev, cin_pad=None, dgrad=False)
        # ---- decoder (forward + input-gradient)
        rch = tuple(reversed(ch))
        self.post_quant = Conv(sd["post_quant_conv.weight"], sd["post_quant_conv.bias"], dev, cin_pad=8,
                               dgrad_rows=list(range(lc)), dgrad_cout_pad=8)
        self.dec_in = Conv(sd["decoder.conv_in.weight"], sd["decoder.conv_in.bias"], dev, cin_pad=8,
                           dgrad_rows=list(range(lc)))
        self.dec_mid = self._mid(sd, "decoder.mid_block.", dev, rch[0], True)
        self.dec_blocks = []
        prev = rch[0]
        for i, c in enumerate(rch):
            res = [_Res(sd, f"decoder.up_blocks.{i}.resnets.{j}.", dev, prev if j == 0 else c, c, True)
                   for j in range(L + 1)]
            up = None
            if i < len(rch) - 1:
                up = Conv(sd[f"decoder.up_blocks.{i}.upsamplers.0.conv.weight"],
                          sd[f"decoder.up_blocks.{i}.upsamplers.0.conv.bias"], dev)
            self.dec_blocks.append((res, up))
            prev = c
        self.dec_norm = Norm(sd["decoder.conv_norm_out.weight"], sd["decoder.conv_norm_out.bias"], dev, 1e-6)
        # conv_out with the output mapped [-1, 1] -> [0, 1] ((y + 1) / 2: weights / 2, bias (b + 1) / 2), the
        # range of TAESD's DecoderTiny output before AutoencoderTiny.decode's "* 2 - 1", which the shared decode
        # tail of the guidance kernels applies (decode_prediction, marigold_dc.py:366)
        self.dec_out = Conv(sd["decoder.conv_out.weight"].float() / 2, (sd["decoder.conv_out.bias"].float() + 1) / 2,
                            dev, dgrad_cout_pad=8)

    @staticmethod
    def _mid(sd, pre, dev, c, dgrad):
        return (_Res(sd, pre + "resnets.0.", dev, c, c, dgrad), _Attn(sd, pre + "attentions.0.", dev, c, dgrad),
                _Res(sd, pre + "resnets.1.", dev, c, c, dgrad))

    def decoder_plan(self, ctx: Ctx, nb: int, h: int, w: int) -> "KLPlan":
        return KLPlan(self, ctx, nb, h, w, decoder=True)

    def encode(self, ctx: Ctx, img8: torch.Tensor, nb: int, H: int, W: int, out):
        """img8 [nb*H*W][8] (the preprocessed image in [-1, 1], channels 0..2) -> the scaled posterior mean
        into `out` (4 channels; marigold_dc.py:696-698)."""
        plan = KLPlan(self, ctx, nb, H, W, decoder=False, enc_in=img8, enc_out=out)
        plan.forward()
        return plan.H, plan.W


class KLPlan:
    """Static buffers + launch lists of the KL encoder (forward) or decoder (forward and input-gradient).
    Decoder: ``tin`` [P][8] (z / scaling_factor in 0..3), ``out`` [P_img][8] ((decoder output + 1) / 2 in
    0..2, the convention of taesd.DecoderPlan), ``dout`` its gradient, ``dtin`` [P][8] the gradient of ``tin``."""

    def __init__(self, net: AutoencoderKLHIP, ctx: Ctx, nb: int, h: int, w: int, decoder: bool, enc_in=None,
                 enc_out=None):
        self.net, self.ctx, self.nb, self.dev = net, ctx, nb, net.device
        self.saved = []
        self.fwd, self.tape = [], []
        if decoder:
            self._build_decoder(h, w)
        else:
            self._build_encoder(h, w, enc_in, enc_out)

    def buf(self, rows, cols, dtype=BF16):
        t = torch.zeros(rows, cols, dtype=dtype, device=self.dev)
        self.saved.append(t)
        return t

    # ------------------------------------------------------------------ blocks (forward)
    def _conv(self, cv: Conv, x, cin, hw, cout, y, ohw=None, mode=0, stride=1, pad=None, resid=None, act=0):
        ctx, nb = self.ctx, self.nb
        hh, ww = hw
        ho, wo = ohw or hw
        k = cv.kh
        pad = (k // 2) if pad is None else pad

        def f():
            ops.conv_gemm(ctx, x, cv.wf, nb=nb, hin=hh, win=ww, cin=cin, hout=ho, wout=wo, cout=cout, kh=k, kw=k,
                          stride=stride, pad=pad, mode=mode, bias=cv.bias, resid=resid, act=act, y=y)

        self.fwd.append(f)

    def _resnet(self, r: _Res, x, hw):
        ctx, nb = self.ctx, self.nb
        hh, ww = hw
        P = nb * hh * ww
        g1, h1, g2, out = self.buf(P, r.cin), self.buf(P, r.cout), self.buf(P, r.cout), self.buf(P, r.cout)
        st1, st2 = self.buf(nb, 64, torch.float32), self.buf(nb, 64, torch.float32)
        sc = self.buf(P, r.cout) if r.shortcut is not None else None

        def f():
            ops.groupnorm(ctx, x, nb, hh * ww, r.cin, r.norm1.gamma, r.norm1.beta, r.norm1.eps, True, g1, st1)
            ops.conv_gemm(ctx, g1, r.conv1.wf, nb=nb, hin=hh, win=ww, cin=r.cin, hout=hh, wout=ww, cout=r.cout,
                          bias=r.conv1.bias, y=h1)
            ops.groupnorm(ctx, h1, nb, hh * ww, r.cout, r.norm2.gamma, r.norm2.beta, r.norm2.eps, True, g2, st2)
            res = x
            if r.shortcut is not None:
                ops.conv_gemm(ctx, x, r.shortcut.wf, nb=nb, hin=hh, win=ww, cin=r.cin, hout=hh, wout=ww,
                              cout=r.cout, kh=1, kw=1, pad=0, bias=r.shortcut.bias, y=sc)
                res = sc
            ops.conv_gemm(ctx, g2, r.conv2.wf, nb=nb, hin=hh, win=ww, cin=r.cout, hout=hh, wout=ww, cout=r.cout,
                          bias=r.conv2.bias, resid=res, y=out)

        self.fwd.append(f)
        self.tape.append(("resnet", dict(r=r, x=x, hw=hw, st1=st1, h1=h1, st2=st2, out=out)))
        return out

    def _attn(self, a: _Attn, x, hw):
        ctx, nb = self.ctx, self.nb
        hh, ww = hw
        T = hh * ww
        Tp = -(-T // 64) * 64
        P, C = nb * T, a.c
        n0, q, k, v, o, out = (self.buf(P, C) for _ in range(6))
        st0 = self.buf(nb, 64, torch.float32)
        pm = self.buf(nb * T, Tp)                  # softmax probabilities, kept for the backward
        s = self.scratch(T, Tp)
        vt = self.scratch_t(C, Tp)
        scale = 1.0 / math.sqrt(C)

        def f():
            ops.groupnorm(ctx, x, nb, T, C, a.norm.gamma, a.norm.beta, a.norm.eps, False, n0, st0)
            ops.linear(ctx, n0, a.q.wf, P, C, q, bias=a.q.bias)
            ops.linear(ctx, n0, a.k.wf, P, C, k, bias=a.k.bias)
            ops.linear(ctx, n0, a.v.wf, P, C, v, bias=a.v.bias)
            for fr in range(nb):
                rs = slice(fr * T, (fr + 1) * T)
                ops.linear(ctx, q[rs], k[rs], T, T, s)                                     # S = Q K^T
                _lib.call("dc_softmax_rows", s.data_ptr(), Tp, T, T, scale, pm[rs].data_ptr(), Tp, ctx.stream)
                _lib.call("dc_transpose", v[rs].data_ptr(), C, T, C, vt.data_ptr(), Tp, ctx.stream)
                ops.linear(ctx, pm[rs], vt, T, C, o[rs])                                   # O = P V
            ops.linear(ctx, o, a.o.wf, P, C, out, bias=a.o.bias, resid=x)

        self.fwd.append(f)
        self.tape.append(("attn", dict(a=a, x=x, hw=hw, st0=st0, n0=n0, q=q, k=k, v=v, pm=pm, out=out, T=T, Tp=Tp)))
        return out

    def scratch(self, rows, cols):
        """[rows][cols] bf16 scratch shared by every attention of the plan (re-used in the backward)."""
        key = ("s", rows, cols)
        if not hasattr(self, "_scr"):
            self._scr = {}
        if key not in self._scr:
            self._scr[key] = [self.buf(rows, cols) for _ in range(3)]
        return self._scr[key][0]

    def scratch_t(self, rows, cols, i=0):
        key = ("t", rows, cols)
        if not hasattr(self, "_scr"):
            self._scr = {}
        if key not in self._scr:
            self._scr[key] = [self.buf(rows, cols) for _ in range(3)]
        return self._scr[key][i]

    def _mid(self, mid, x, hw):
        x = self._resnet(mid[0], x, hw)
        x = self._attn(mid[1], x, hw)
        return self._resnet(mid[2], x, hw)

    # ------------------------------------------------------------------ encoder
    def _build_encoder(self, H, W, img8, out):
        net, nb = self.net, self.nb
        ch = net.cfg.block_out_channels
        hw = (H, W)
        x = self.buf(nb * H * W, ch[0])
        self._conv(net.enc_in, img8, 8, hw, ch[0], x)
        for res, down in net.enc_blocks:
            for r in res:
                x = self._resnet(r, x, hw)
            if down is not None:
                ho, wo = (hw[0] - 2) // 2 + 1, (hw[1] - 2) // 2 + 1   # F.pad (0, 1, 0, 1) + conv s2 p0
                y = self.buf(nb * ho * wo, down.cout)
                self._conv(down, x, down.cin, hw, down.cout, y, ohw=(ho, wo), stride=2, pad=0)
                x, hw = y, (ho, wo)
        x = self._mid(net.enc_mid, x, hw)
        P = nb * hw[0] * hw[1]
        g, st = self.buf(P, ch[-1]), self.buf(nb, 64, torch.float32)
        e = self.buf(P, 8)
        n = net.enc_norm

        def f(x=x, g=g, st=st, hh=hw[0], ww=hw[1]):
            ops.groupnorm(self.ctx, x, nb, hh * ww, ch[-1], n.gamma, n.beta, n.eps, True, g, st)

        self.fwd.append(f)
        self._conv(net.enc_out, g, ch[-1], hw, 8, e)
        self._conv(net.quant, e, 8, hw, net.cfg.latent_channels, out)
        self.H, self.W = hw

    # ------------------------------------------------------------------ decoder
    def _build_decoder(self, h, w):
        net, nb, ctx = self.net, self.nb, self.ctx
        rch = tuple(reversed(net.cfg.block_out_channels))
        lc = net.cfg.latent_channels
        hw = (h, w)
        P = nb * h * w
        self.tin = self.buf(P, 8)
        self.dtin = self.buf(P, 8)
        pq = self.buf(P, 8)
        self._conv(net.post_quant, self.tin, 8, hw, lc, pq)
        x0 = self.buf(P, rch[0])
        self._conv(net.dec_in, pq, 8, hw, rch[0], x0)
        x = self._mid(net.dec_mid, x0, hw)
        for res, up in net.dec_blocks:
            for r in res:
                x = self._resnet(r, x, hw)
            if up is not None:
                ohw = (2 * hw[0], 2 * hw[1])
                y = self.buf(nb * ohw[0] * ohw[1], up.cout)
                self._conv(up, x, up.cin, hw, up.cout, y, ohw=ohw, mode=1)
                self.tape.append(("up", dict(cv=up, x=x, hw=hw, ohw=ohw, out=y)))
                x, hw = y, ohw
        self.H, self.W = hw
        Pi = nb * hw[0] * hw[1]
        c = rch[-1]
        g, st = self.buf(Pi, c), self.buf(nb, 64, torch.float32)
        n = net.dec_norm
        xl = x

        def fn(hh=hw[0], ww=hw[1]):
            ops.groupnorm(ctx, xl, nb, hh * ww, c, n.gamma, n.beta, n.eps, True, g, st)

        self.fwd.append(fn)
        self.out = self.buf(Pi, 8)
        self.dout = self.buf(Pi, 8)
        self._conv(net.dec_out, g, c, hw, 3, self.out)
        # ---- backward (input-gradient only), reverse order
        bwd = []
        dg = self.buf(Pi, c)
        dx = self.buf(Pi, c)

        def b_out(hh=hw[0], ww=hw[1]):
            ops.conv_gemm(ctx, self.dout, net.dec_out.wd, nb=nb, hin=hh, win=ww, cin=8, hout=hh, wout=ww, cout=c,
                          y=dg)
            ops.groupnorm_bwd(ctx, xl, nb, hh * ww, c, n.gamma, n.beta, True, st, dg, dx)

        bwd.append(b_out)
        grad = {id(xl): dx}
        for kind, d in reversed(self.tape):
            gout = grad[id(d["out"])]
            if kind == "resnet":
                bwd.append(self._resnet_bwd(d, gout, grad))
            elif kind == "attn":
                bwd.append(self._attn_bwd(d, gout, grad))
            else:
                bwd.append(self._up_bwd(d, gout, grad))
        gx0 = grad[id(x0)]
        dpq = self.buf(P, 8)

        def b_in():
            ops.conv_gemm(ctx, gx0, net.dec_in.wd, nb=nb, hin=h, win=w, cin=rch[0], hout=h, wout=w, cout=lc, y=dpq)
            ops.conv_gemm(ctx, dpq, net.post_quant.wd, nb=nb, hin=h, win=w, cin=8, hout=h, wout=w, cout=lc, kh=1,
                          kw=1, pad=0, y=self.dtin)

        bwd.append(b_in)
        self.bwd = bwd

    def _resnet_bwd(self, d, dout, grad):
        ctx, nb = self.ctx, self.nb
        r, x, (hh, ww) = d["r"], d["x"], d["hw"]
        st1, h1, st2 = d["st1"], d["h1"], d["st2"]
        P = nb * hh * ww
        dg2, dh1, dg1, dx = self.buf(P, r.cout), self.buf(P, r.cout), self.buf(P, r.cin), self.buf(P, r.cin)
        grad[id(x)] = dx

        def b():
            kw = dict(nb=nb, hin=hh, win=ww, hout=hh, wout=ww)
            ops.conv_gemm(ctx, dout, r.conv2.wd, cin=r.cout, cout=r.cout, y=dg2, **kw)
            ops.groupnorm_bwd(ctx, h1, nb, hh * ww, r.cout, r.norm2.gamma, r.norm2.beta, True, st2, dg2, dh1)
            ops.conv_gemm(ctx, dh1, r.conv1.wd, cin=r.cout, cout=r.cin, y=dg1, **kw)
            if r.shortcut is None:
                ops.groupnorm_bwd(ctx, x, nb, hh * ww, r.cin, r.norm1.gamma, r.norm1.beta, True, st1, dg1, dx,
                                  add1=dout)
            else:
                ops.groupnorm_bwd(ctx, x, nb, hh * ww, r.cin, r.norm1.gamma, r.norm1.beta, True, st1, dg1, dx)
                ops.conv_gemm(ctx, dout, r.shortcut.wd, cin=r.cout, cout=r.cin, kh=1, kw=1, pad=0, resid=dx, y=dx,
                              **kw)

        return b

    def _attn_bwd(self, d, dout, grad):
        ctx, nb = self.ctx, self.nb
        a, x, st0, n0 = d["a"], d["x"], d["st0"], d["n0"]
        q, k, v, pm, T, Tp = d["q"], d["k"], d["v"], d["pm"], d["T"], d["Tp"]
        C = a.c
        P = nb * T
        do, dq, dk, dv, dn, dx = (self.buf(P, C) for _ in range(6))
        grad[id(x)] = dx
        self.scratch(T, Tp)
        sbuf = self._scr[("s", T, Tp)]
        tbuf = [self.scratch_t(C, Tp, i) for i in range(3)]
        scale = 1.0 / math.sqrt(C)

        def b():
            dp_, ds_, dst_ = sbuf
            ops.linear(ctx, dout, a.o.wd, P, C, do)                                        # dO
            for fr in range(nb):
                rs = slice(fr * T, (fr + 1) * T)
                ops.linear(ctx, do[rs], v[rs], T, T, dp_)                                  # dP = dO V^T
                _lib.call("dc_softmax_rows_bwd", pm[rs].data_ptr(), Tp, dp_.data_ptr(), Tp, T, T, scale,
                          ds_.data_ptr(), Tp, ctx.stream)
                _lib.call("dc_transpose", k[rs].data_ptr(), C, T, C, tbuf[0].data_ptr(), Tp, ctx.stream)
                ops.linear(ctx, ds_, tbuf[0], T, C, dq[rs])                                # dQ = dS K
                _lib.call("dc_transpose", ds_.data_ptr(), Tp, T, T, dst_.data_ptr(), Tp, ctx.stream)
                _lib.call("dc_transpose", q[rs].data_ptr(), C, T, C, tbuf[1].data_ptr(), Tp, ctx.stream)
                ops.linear(ctx, dst_, tbuf[1], T, C, dk[rs])                               # dK = dS^T Q
                _lib.call("dc_transpose", pm[rs].data_ptr(), Tp, T, T, dst_.data_ptr(), Tp, ctx.stream)
                _lib.call("dc_transpose", do[rs].data_ptr(), C, T, C, tbuf[2].data_ptr(), Tp, ctx.stream)
                ops.linear(ctx, dst_, tbuf[2], T, C, dv[rs])                               # dV = P^T dO
            ops.linear(ctx, dq, a.q.wd, P, C, dn)
            ops.linear(ctx, dk, a.k.wd, P, C, dn, resid=dn)
            ops.linear(ctx, dv, a.v.wd, P, C, dn, resid=dn)
            ops.groupnorm_bwd(ctx, x, nb, T, C, a.norm.gamma, a.norm.beta, False, st0, dn, dx, add1=dout)

        return b

    def _up_bwd(self, d, dout, grad):
        ctx, nb = self.ctx, self.nb
        cv, x, (hh, ww), (ho, wo) = d["cv"], d["x"], d["hw"], d["ohw"]
        dhi = self.buf(nb * ho * wo, cv.cin)
        dlo = self.buf(nb * hh * ww, cv.cin)
        grad[id(x)] = dlo

        def b():
            ops.conv_gemm(ctx, dout, cv.wd, nb=nb, hin=ho, win=wo, cin=cv.cout, hout=ho, wout=wo, cout=cv.cin, y=dhi)
            ops.upsample_adjoint(ctx, dhi, nb, ho, wo, cv.cin, hh, ww, dlo)

        return b

    def set_rows(self, rows):
        """Dense only: the decoder's GroupNorms need whole-map statistics, so no sparse-aware decode."""
        if rows is not None:
            raise ValueError("AutoencoderKL decoder plan has no row-list mode")

    def forward(self):
        for f in self.fwd:
            f()
        return getattr(self, "out", None)

    def backward(self):
        for b in self.bwd:
            b()
        return self.dtin

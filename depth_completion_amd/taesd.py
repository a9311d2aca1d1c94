"""TAESD (diffusers AutoencoderTiny, ``madebyollin/taesd``) encoder / decoder on HIP kernels.

Decoder forward + input-gradient replace ``decode_prediction`` -> ``vae.decode`` inside
``_latent_to_affine`` (marigold_dc.py:366) and its part of ``losses.backward`` (:877); the
encoder replaces ``prepare_latents`` -> ``vae.encode`` (marigold_dc.py:696-698), once per call.
DecoderTiny: tanh(x/3)*3 -> conv(4->64)+ReLU -> 3 blocks -> [up2x, conv, 3 blocks] x2 ->
[up2x, conv, 1 block] -> conv(64->3); block(x) = relu(conv(relu(conv(relu(conv(x))))) + x).
"""
from __future__ import annotations

import torch

from . import ops
from .ops import BF16, Ctx
from .weights import Conv

DEC_BLOCKS = (3, 3, 3, 1)
ENC_BLOCKS = (1, 3, 3, 3)
CH = 64


class TAESDHIP:
    def __init__(self, sd: dict, device):
        dev = torch.device(device)
        self.device = dev
        self.dec = []  # list of ("conv", Conv, act) / ("block", [Conv]*3) / ("up",) / ("up_conv", Conv)
        i = 0
        self.dec_in = Conv(sd[f"decoder.layers.{i}.weight"], sd[f"decoder.layers.{i}.bias"], dev, cin_pad=8,
                           dgrad_rows=[0, 1, 2, 3])
        i = 2
        for bi, nblk in enumerate(DEC_BLOCKS):
            for _ in range(nblk):
                convs = [Conv(sd[f"decoder.layers.{i}.conv.{k}.weight"], sd[f"decoder.layers.{i}.conv.{k}.bias"], dev)
                         for k in (0, 2, 4)]
                self.dec.append(("block", convs))
                i += 1
            if bi < len(DEC_BLOCKS) - 1:
                i += 1  # nn.Upsample
                self.dec.append(("up_conv", Conv(sd[f"decoder.layers.{i}.weight"], None, dev)))
                i += 1
        self.dec_out = Conv(sd[f"decoder.layers.{i}.weight"], sd[f"decoder.layers.{i}.bias"], dev, dgrad_cout_pad=8)
        # encoder (forward only)
        self.enc = []
        i = 0
        for bi, nblk in enumerate(ENC_BLOCKS):
            if bi == 0:
                self.enc.append(("conv", Conv(sd[f"encoder.layers.{i}.weight"], sd[f"encoder.layers.{i}.bias"], dev,
                                              cin_pad=8, dgrad=False)))
            else:
                self.enc.append(("down", Conv(sd[f"encoder.layers.{i}.weight"], None, dev, stride=2, dgrad=False)))
            i += 1
            for _ in range(nblk):
                convs = [Conv(sd[f"encoder.layers.{i}.conv.{k}.weight"], sd[f"encoder.layers.{i}.conv.{k}.bias"], dev,
                              dgrad=False) for k in (0, 2, 4)]
                self.enc.append(("block", convs))
                i += 1
        self.enc_out = Conv(sd[f"encoder.layers.{i}.weight"], sd[f"encoder.layers.{i}.bias"], dev, dgrad=False)

    def decoder_plan(self, ctx: Ctx, nb: int, h: int, w: int) -> "DecoderPlan":
        return DecoderPlan(self, ctx, nb, h, w)

    def encode(self, ctx: Ctx, img8: torch.Tensor, nb: int, H: int, W: int, out, out_ld_view=None):
        """img8 [nb*H*W][8] (EncoderTiny input, already mapped to [0,1]) -> latents into `out` (4 channels)."""
        dev = self.device
        hh, ww = H, W
        x = img8
        keep = []
        for kind, cv in self.enc:
            if kind == "conv":
                y = torch.empty(nb * hh * ww, CH, dtype=BF16, device=dev)
                ops.conv_gemm(ctx, x, cv.wf, nb=nb, hin=hh, win=ww, cin=8, hout=hh, wout=ww, cout=CH, bias=cv.bias, y=y)
            elif kind == "down":
                ho, wo = (hh - 1) // 2 + 1, (ww - 1) // 2 + 1
                y = torch.empty(nb * ho * wo, CH, dtype=BF16, device=dev)
                ops.conv_gemm(ctx, x, cv.wf, nb=nb, hin=hh, win=ww, cin=CH, hout=ho, wout=wo, cout=CH, stride=2, y=y)
                hh, ww = ho, wo
            else:
                y = self._block_fwd(ctx, cv, x, nb, hh, ww, keep)
            keep.append(y)
            x = y
        ops.conv_gemm(ctx, x, self.enc_out.wf, nb=nb, hin=hh, win=ww, cin=CH, hout=hh, wout=ww, cout=4,
                      bias=self.enc_out.bias, y=out)
        return hh, ww

    def _block_fwd(self, ctx, convs, x, nb, hh, ww, keep, bufs=None):
        dev = self.device
        P = nb * hh * ww
        a1, a2, o = bufs if bufs is not None else [torch.empty(P, CH, dtype=BF16, device=dev) for _ in range(3)]
        kw = dict(nb=nb, hin=hh, win=ww, cin=CH, hout=hh, wout=ww, cout=CH)
        ops.conv_gemm(ctx, x, convs[0].wf, bias=convs[0].bias, act=1, y=a1, **kw)
        ops.conv_gemm(ctx, a1, convs[1].wf, bias=convs[1].bias, act=1, y=a2, **kw)
        ops.conv_gemm(ctx, a2, convs[2].wf, bias=convs[2].bias, resid=x, act=1, y=o, **kw)
        keep.extend([a1, a2])
        return o


class DecoderPlan:
    """Static buffers + launch lists of DecoderTiny forward and input-gradient for (nb, h, w) latents.
    ``tin`` [P][8]: clamp(x0) input (0..3); ``out`` [P_img][8]: decoder output (0..2);
    ``dout`` [P_img][8]: its gradient; ``dtin`` [P][8]: gradient of ``tin`` (0..3)."""

    def __init__(self, net: TAESDHIP, ctx: Ctx, nb: int, h: int, w: int):
        self.net, self.ctx, self.nb = net, ctx, nb
        dev = net.device
        self.saved = []
        # sparse-aware mode (set_rows): the full-resolution convs run on row lists -- S0 the resize taps of
        # the sparse pixels, S(k+1) = S(k) dilated by 3x3 -- keyed by launch: out S0, c3 / bfin S1,
        # c2 / dc2 S2, c1 / dc1 S3, up / dx S4, dhi S5
        self.rows = None
        self._full_res_grads = []

        def R(key, full):
            return self.rows[key] if (self.rows is not None and full) else None

        def buf(rows, cols=CH):
            t = torch.zeros(rows, cols, dtype=BF16, device=dev)
            self.saved.append(t)
            return t

        self.tin = buf(nb * h * w, 8)
        self.dtin = buf(nb * h * w, 8)
        fwd, tape = [], []
        hh, ww = h, w
        a0 = buf(nb * hh * ww)
        tin = self.tin

        def f0(a0=a0, hh=hh, ww=ww):
            ops.conv_gemm(ctx, tin, net.dec_in.wf, nb=nb, hin=hh, win=ww, cin=8, hout=hh, wout=ww, cout=CH,
                          bias=net.dec_in.bias, act=1, y=a0)

        fwd.append(f0)
        x, x_is_relu = a0, True
        for kind, cv in net.dec:
            P = nb * hh * ww
            if kind == "block":
                a1, a2, o = buf(P), buf(P), buf(P)

                def fb(cv=cv, x=x, a1=a1, a2=a2, o=o, hh=hh, ww=ww):
                    kw = dict(nb=nb, hin=hh, win=ww, cin=CH, hout=hh, wout=ww, cout=CH)
                    full = (hh, ww) == (self.H, self.W)
                    ops.conv_gemm(ctx, x, cv[0].wf, bias=cv[0].bias, act=1, y=a1, rows=R("c1", full), **kw)
                    ops.conv_gemm(ctx, a1, cv[1].wf, bias=cv[1].bias, act=1, y=a2, rows=R("c2", full), **kw)
                    ops.conv_gemm(ctx, a2, cv[2].wf, bias=cv[2].bias, resid=x, act=1, y=o, rows=R("c3", full), **kw)

                fwd.append(fb)
                tape.append(("block", dict(cv=cv, x=x, x_relu=x_is_relu, a1=a1, a2=a2, o=o, hw=(hh, ww))))
                x, x_is_relu = o, True
            else:  # up_conv
                ho, wo = 2 * hh, 2 * ww
                y = buf(nb * ho * wo)

                def fu(cv=cv, x=x, y=y, hh=hh, ww=ww, ho=ho, wo=wo):
                    ops.conv_gemm(ctx, x, cv.wf, nb=nb, hin=hh, win=ww, cin=CH, hout=ho, wout=wo, cout=CH, mode=1, y=y,
                                  rows=R("up", (ho, wo) == (self.H, self.W)))

                fwd.append(fu)
                tape.append(("up_conv", dict(cv=cv, x=x, x_relu=x_is_relu, y=y, hw=(hh, ww), ohw=(ho, wo))))
                x, x_is_relu = y, False
                hh, ww = ho, wo
        self.H, self.W = hh, ww
        self.out = buf(nb * hh * ww, 8)
        self.dout = buf(nb * hh * ww, 8)
        xl = x

        def ff(hh=hh, ww=ww):
            ops.conv_gemm(ctx, xl, net.dec_out.wf, nb=nb, hin=hh, win=ww, cin=CH, hout=hh, wout=ww, cout=3,
                          bias=net.dec_out.bias, y=self.out, rows=R("out", True))

        fwd.append(ff)
        self.fwd = fwd
        # ---- backward
        bwd = []
        P = nb * hh * ww
        dpre = buf(P)   # grad w.r.t. the pre-ReLU fuse of the last block
        last_is_relu = x_is_relu

        def bfin(dpre=dpre, hh=hh, ww=ww):
            ops.conv_gemm(ctx, self.dout, net.dec_out.wd, nb=nb, hin=hh, win=ww, cin=8, hout=hh, wout=ww, cout=CH,
                          mask=xl if last_is_relu else None, y=dpre, rows=R("c3", True))

        self._full_res_grads.append(dpre)

        bwd.append(bfin)
        g = dpre  # gradient w.r.t. the (pre-activation) value feeding `x`
        for kind, d in reversed(tape):
            if kind == "block":
                cv, x, a1, a2 = d["cv"], d["x"], d["a1"], d["a2"]
                hh, ww = d["hw"]
                P = nb * hh * ww
                dc2, dc1, dx = buf(P), buf(P), buf(P)
                if (hh, ww) == (self.H, self.W):
                    self._full_res_grads += [dc2, dc1, dx]

                def bb(cv=cv, g=g, x=x, a1=a1, a2=a2, dc2=dc2, dc1=dc1, dx=dx, hh=hh, ww=ww, xr=d["x_relu"]):
                    kw = dict(nb=nb, hin=hh, win=ww, cin=CH, hout=hh, wout=ww, cout=CH)
                    full = (hh, ww) == (self.H, self.W)
                    ops.conv_gemm(ctx, g, cv[2].wd, mask=a2, y=dc2, rows=R("c2", full), **kw)
                    ops.conv_gemm(ctx, dc2, cv[1].wd, mask=a1, y=dc1, rows=R("c1", full), **kw)
                    ops.conv_gemm(ctx, dc1, cv[0].wd, resid=g, mask=x if xr else None, y=dx, rows=R("up", full), **kw)

                bwd.append(bb)
                g = dx
            else:
                cv, x = d["cv"], d["x"]
                hh, ww = d["hw"]
                ho, wo = d["ohw"]
                dhi = buf(nb * ho * wo)
                dlo = buf(nb * hh * ww)
                if (ho, wo) == (self.H, self.W):
                    self._full_res_grads.append(dhi)

                def bu(cv=cv, g=g, x=x, dhi=dhi, dlo=dlo, hh=hh, ww=ww, ho=ho, wo=wo, xr=d["x_relu"]):
                    ops.conv_gemm(ctx, g, cv.wd, nb=nb, hin=ho, win=wo, cin=CH, hout=ho, wout=wo, cout=CH, y=dhi,
                                  rows=R("dhi", (ho, wo) == (self.H, self.W)))
                    ops.upsample_adjoint(ctx, dhi, nb, ho, wo, CH, hh, ww, dlo, mask=x if xr else None)

                bwd.append(bu)
                g = dlo
        g0 = g  # gradient w.r.t. relu(conv0) pre-activation (already masked by a0)

        def b0():
            ops.conv_gemm(ctx, g0, net.dec_in.wd, nb=nb, hin=h, win=w, cin=CH, hout=h, wout=w, cout=4, y=self.dtin)

        bwd.append(b0)
        self.bwd = bwd

    def set_rows(self, rows):
        """rows: None (dense) or {"out", "c3", "c2", "c1", "up", "dhi"} -> (int32 row list, count) for the
        sets S0, S1, S2, S3, S4, S5 of the full-resolution level.  The gradient buffers of that level are
        zeroed, as the sparse backward writes only inside the sets and reads its neighbours."""
        self.rows = rows
        if rows is not None:
            for t in self._full_res_grads:
                ops.memset(self.ctx, t)

    def forward(self):
        for f in self.fwd:
            f()
        return self.out

    def backward(self):
        for b in self.bwd:
            b()
        return self.dtin

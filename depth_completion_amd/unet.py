"""UNet2DConditionModel (Marigold v1-0, SD2 architecture) forward + input-gradient on HIP kernels.

Replaces ``self.unet(...)`` in ``_predict_noise`` (marigold_dc.py:459-465) and the UNet part of
``losses.backward`` (marigold_dc.py:877).  A ``UNetPlan`` is built once per (frames, latent h, w):
all activations, saved tensors and gradient buffers are allocated up front (NHWC pixel rows), and
the forward / backward are flat lists of kernel launches with bound pointers -- the shape a
hipGraph capture of one guided step needs.  Only the gradient w.r.t. the depth-latent half of the
8-channel input is produced (the image-latent half and all weights are constants).
"""
from __future__ import annotations

import os

import torch

from . import ops
from .config import UNetConfig
from .ops import BF16, Ctx, Slice
from .weights import Conv, FoldedPair, Linear, LnLinear, Norm, fold_cross_attention, geglu_interleave, round_bf16


class ResnetW:
    def __init__(self, sd, pre, dev):
        self.norm1 = Norm(sd[pre + "norm1.weight"], sd[pre + "norm1.bias"], dev, 1e-5)
        self.conv1 = Conv(sd[pre + "conv1.weight"], sd[pre + "conv1.bias"], dev)
        self.temb_w = sd[pre + "time_emb_proj.weight"]
        self.temb_b = sd[pre + "time_emb_proj.bias"]
        self.temb = Linear(self.temb_w, self.temb_b, dev, dgrad=False)
        self.norm2 = Norm(sd[pre + "norm2.weight"], sd[pre + "norm2.bias"], dev, 1e-5)
        self.conv2 = Conv(sd[pre + "conv2.weight"], sd[pre + "conv2.bias"], dev)
        self.cin = self.conv1.cin
        self.cout = self.conv1.cout
        self.shortcut = None
        if pre + "conv_shortcut.weight" in sd:
            self.shortcut = Conv(sd[pre + "conv_shortcut.weight"], sd[pre + "conv_shortcut.bias"], dev)
        self.temb_table = None  # [S][cout] bf16: the current call's entry of temb_tables
        # one table per step count, never freed: a captured step graph binds the table's address, and a
        # call with another step count must not free the one an earlier graph replays against
        self.temb_tables: dict = {}


def ff_fold_enabled() -> bool:
    """FF2 and proj_out folded into one two-source linear (include/dcamd.h dc_fold_linear_pair; forward and input-
    gradient one launch each instead of two); DC_FF_FOLD=0: the two linears, for A/B runs and tests -- the native
    session always folds."""
    return os.environ.get("DC_FF_FOLD", "1") != "0"


def ln_fuse_enabled() -> bool:
    """LayerNorm norm3 folded into ff.net.0.proj (include/dcamd.h dc_ln_fuse: its statistics from the cross-attention
    kernel that produces its input) and its backward into the cross-attention backward; DC_LN_FUSE=0: the separate
    LayerNorm launches, for A/B runs and tests -- the native session always folds."""
    return os.environ.get("DC_LN_FUSE", "1") != "0"


class TransformerW:
    def __init__(self, sd, pre, dev, heads, ctx):
        self.heads = heads
        self.ln_fused = ln_fuse_enabled()
        self.norm = Norm(sd[pre + "norm.weight"], sd[pre + "norm.bias"], dev, 1e-6)
        self.proj_in = Linear(sd[pre + "proj_in.weight"], sd[pre + "proj_in.bias"], dev)
        b = pre + "transformer_blocks.0."
        self.ln1 = Norm(sd[b + "norm1.weight"], sd[b + "norm1.bias"], dev, 1e-5)
        self.ln2 = Norm(sd[b + "norm2.weight"], sd[b + "norm2.bias"], dev, 1e-5)
        self.ln3 = Norm(sd[b + "norm3.weight"], sd[b + "norm3.bias"], dev, 1e-5)
        wqkv = torch.cat([sd[b + "attn1.to_q.weight"], sd[b + "attn1.to_k.weight"], sd[b + "attn1.to_v.weight"]], 0)
        self.qkv = Linear(wqkv, None, dev)
        self.out = Linear(sd[b + "attn1.to_out.0.weight"], sd[b + "attn1.to_out.0.bias"], dev)
        U, D, c0 = fold_cross_attention(sd, b + "attn2.", ctx, heads)
        self.U, self.D, self.c0 = U.to(dev), D.to(dev), c0.to(dev)
        self.cross_tabs = None  # MFMA operand tables (ops.crossattn_tables), built with the first context
        # GEGLU projection with (h, gate) rows interleaved 8 + 8 for the fused epilogues (geglu_interleave)
        perm = geglu_interleave(sd[b + "ff.net.0.proj.weight"].shape[0])
        if self.ln_fused:   # norm3 folded into ff.net.0.proj
            self.ff1 = LnLinear(sd[b + "ff.net.0.proj.weight"][perm], sd[b + "ff.net.0.proj.bias"][perm],
                                sd[b + "norm3.weight"], sd[b + "norm3.bias"], 1e-5, dev)
        else:
            self.ff1 = Linear(sd[b + "ff.net.0.proj.weight"][perm], sd[b + "ff.net.0.proj.bias"][perm], dev)
        self.c = self.proj_in.cout
        self.ffo = self.ff2 = self.proj_out = None
        if ff_fold_enabled():   # FF2 + proj_out as one linear over [gg | r2]
            self.ffo = FoldedPair(sd[b + "ff.net.2.weight"], sd[b + "ff.net.2.bias"], sd[pre + "proj_out.weight"],
                                  sd[pre + "proj_out.bias"], dev)
        else:
            self.ff2 = Linear(sd[b + "ff.net.2.weight"], sd[b + "ff.net.2.bias"], dev)
            self.proj_out = Linear(sd[pre + "proj_out.weight"], sd[pre + "proj_out.bias"], dev)


def timestep_embedding(timesteps: torch.Tensor, dim: int) -> torch.Tensor:
    """diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0), fp32, host: the library's
    dc_timestep_embedding, which the native session (csrc/session.cpp) uses too (same bits on both hosts)."""
    from . import _lib
    ts = timesteps.detach().cpu().to(torch.int64).contiguous()
    out = torch.empty(ts.numel(), dim, dtype=torch.float32)
    _lib.call("dc_timestep_embedding", ts.data_ptr(), ts.numel(), dim, out.data_ptr())
    return out


class UNetHIP:
    def __init__(self, sd: dict, cfg: UNetConfig, device, text_embedding: torch.Tensor):
        dev = torch.device(device)
        self.cfg = cfg
        self.device = dev
        ctx = text_embedding.reshape(-1, text_embedding.shape[-1]).float()
        # conv_in: 8 input channels; input-gradient only for channels 4..7 (the depth latent)
        self.conv_in = Conv(sd["conv_in.weight"], sd["conv_in.bias"], dev, dgrad_rows=[4, 5, 6, 7])
        self.t_lin1 = Linear(sd["time_embedding.linear_1.weight"], sd["time_embedding.linear_1.bias"], dev, False)
        self.t_lin2 = Linear(sd["time_embedding.linear_2.weight"], sd["time_embedding.linear_2.bias"], dev, False)
        self.down = []
        nb_ = len(cfg.block_out_channels)
        for i in range(nb_):
            blk = {"resnets": [], "attns": [], "down": None}
            for j in range(cfg.layers_per_block):
                blk["resnets"].append(ResnetW(sd, f"down_blocks.{i}.resnets.{j}.", dev))
                if cfg.down_attn[i]:
                    blk["attns"].append(TransformerW(sd, f"down_blocks.{i}.attentions.{j}.", dev, cfg.heads[i], ctx))
            if i < nb_ - 1:
                blk["down"] = Conv(sd[f"down_blocks.{i}.downsamplers.0.conv.weight"],
                                   sd[f"down_blocks.{i}.downsamplers.0.conv.bias"], dev, stride=2)
            self.down.append(blk)
        self.mid_res = [ResnetW(sd, f"mid_block.resnets.{j}.", dev) for j in range(2)]
        self.mid_attn = TransformerW(sd, "mid_block.attentions.0.", dev, cfg.heads[-1], ctx)
        self.up = []
        rev_heads = list(reversed(cfg.heads))
        for i in range(nb_):
            blk = {"resnets": [], "attns": [], "up": None}
            for j in range(cfg.layers_per_block + 1):
                blk["resnets"].append(ResnetW(sd, f"up_blocks.{i}.resnets.{j}.", dev))
                if cfg.up_attn[i]:
                    blk["attns"].append(TransformerW(sd, f"up_blocks.{i}.attentions.{j}.", dev, rev_heads[i], ctx))
            if i < nb_ - 1:
                blk["up"] = Conv(sd[f"up_blocks.{i}.upsamplers.0.conv.weight"],
                                 sd[f"up_blocks.{i}.upsamplers.0.conv.bias"], dev)
            self.up.append(blk)
        self.norm_out = Norm(sd["conv_norm_out.weight"], sd["conv_norm_out.bias"], dev, 1e-5)
        # conv_out 320->4: forward output padded to ld 8; input-gradient reads dv [P][8] (4..7 zero)
        self.conv_out = Conv(sd["conv_out.weight"], sd["conv_out.bias"], dev, dgrad_cout_pad=8)
        self._temb_key: dict = {}   # step count -> the timesteps its temb tables were built for

    def resnets(self):
        for blk in self.down:
            yield from blk["resnets"]
        yield from self.mid_res
        for blk in self.up:
            yield from blk["resnets"]

    def build_temb_tables(self, ctx: Ctx, timesteps: torch.Tensor):
        """Per-resnet time-embedding projections for every timestep of the call: [S][cout] bf16.

        diffusers: t_emb (fp32) -> bf16 -> linear_1 -> SiLU -> linear_2 (= emb); each resnet adds
        time_emb_proj(SiLU(emb)) to conv1's output (ResnetBlock2D).  Run on the device kernels.
        """
        S = timesteps.shape[0]
        key = tuple(int(t) for t in timesteps.detach().cpu().tolist())
        if self._temb_key.get(S) == key:   # the tables of these timesteps are already built (weights are fixed)
            for r in self.resnets():
                r.temb_table = r.temb_tables[S]
            return
        c0 = self.cfg.block_out_channels[0]
        te = timestep_embedding(timesteps.cpu(), c0).to(BF16).to(self.device)
        d = self.cfg.time_embed_dim
        h1 = torch.empty(S, d, dtype=BF16, device=self.device)
        ops.linear(ctx, te, self.t_lin1.wf, S, d, h1, bias=self.t_lin1.bias)
        a1 = torch.empty_like(h1)
        ops.silu(ctx, h1, a1)
        emb = torch.empty_like(h1)
        ops.linear(ctx, a1, self.t_lin2.wf, S, d, emb, bias=self.t_lin2.bias)
        semb = torch.empty_like(emb)
        ops.silu(ctx, emb, semb)
        for r in self.resnets():
            # one table per step count, kept for the UNet's lifetime (hipGraph replay binds its address)
            if S not in r.temb_tables:
                r.temb_tables[S] = torch.empty(S, r.cout, dtype=BF16, device=self.device)
            r.temb_table = r.temb_tables[S]
            ops.linear(ctx, semb, r.temb.wf, S, r.cout, r.temb_table, bias=r.temb.bias)
        self._temb_key[S] = key

    def plan(self, ctx: Ctx, nb: int, h: int, w: int) -> "UNetPlan":
        return UNetPlan(self, ctx, nb, h, w)


def _conv_out_hw(h, stride):
    return (h + 2 - 3) // stride + 1


class UNetPlan:
    """Buffers + launch lists for one (frames, h, w).  ``x8`` [P][8]: image latents (0..3) and depth
    latents (4..7); ``v`` [P][8]: the v-prediction (0..3); ``dv`` [P][8]: its incoming gradient;
    ``gx`` [P][8]: gradient w.r.t. the depth latents (0..3)."""

    def __init__(self, net: UNetHIP, ctx: Ctx, nb: int, h: int, w: int):
        self.net, self.ctx, self.nb, self.h, self.w = net, ctx, nb, h, w
        dev = net.device
        self.dev = dev
        self.fwd: list = []
        self.tape: list = []          # (kind, info) in forward order
        self.saved: list = []         # keep-alive for every buffer
        P = nb * h * w
        self.x8 = self.buf(P, 8)
        self.v = self.buf(P, 8)
        self.dv = self.buf(P, 8)
        self.gx = self.buf(P, 8)
        # GroupNorm statistics fused into the producing convs (include/dcamd.h dc_gn_fuse; DC_GN_FUSE=0: the
        # separate statistics passes).  One exact accumulator per GroupNorm and direction, all in one arena that
        # the forward zero-fills first; a producer looks up the GroupNorms its output feeds (_gn_targets) at call
        # time, since a skip tensor's up-block consumer is planned long after its producer.
        self.fuse_gn = os.environ.get("DC_GN_FUSE", "1") != "0"
        self.groups = net.cfg.norm_num_groups
        n_res = sum(1 for _ in net.resnets())
        n_tr = sum(len(b["attns"]) for b in net.down + net.up) + 1
        n_gn = 2 * (2 * n_res + n_tr + 1)
        self._gn_words = ops.gn_acc_words(nb, self.groups)
        self.gn_arena = torch.zeros(n_gn * self._gn_words, dtype=torch.int64, device=dev)
        self._gn_slots = n_gn
        self._gn_next = 0
        self._gn_targets: dict = {}   # id(tensor) -> [(acc, coff, groups, cpg, hw)]
        self._gn_fuse: dict = {}      # id(tensor) -> ops.GnFuse, built at the first call
        # the resnet shortcut convs (forward 1x1 and its input-gradient) depend on nothing of their block's main branch
        # (GN -> conv -> GN -> conv).  DC_SIDE_STREAM=1 runs them on a second stream, a fork / join in the captured
        # step graph, to fill CUs the main branch leaves idle at the small levels; measured 5 % slower at C2 (1.733 ->
        # 1.645 fps, ~22 us per fork / join: the graph's cross-queue waits cost more than the overlap returns,
        # profiles/r06p), so one stream is the default.  Same arithmetic either way.
        self.side = ctx.side() if dev.type == "cuda" and os.environ.get("DC_SIDE_STREAM", "0") == "1" else None
        self._build_forward()
        self.bwd: list = []
        self._build_backward()

    # ------------------------------------------------------------------ helpers
    def buf(self, rows, cols, dtype=BF16):
        t = torch.zeros(rows, cols, dtype=dtype, device=self.dev)
        self.saved.append(t)
        return t

    def fbuf(self, *shape):
        t = torch.zeros(*shape, dtype=torch.float32, device=self.dev)
        self.saved.append(t)
        return t

    def _branch(self, fn):
        """fn(ctx) as a branch forked from the current stream (on the side context's stream and workspace); returns
        the join, to be called before the first consumer of the branch's output."""
        if self.side is None:
            fn(self.ctx)
            return lambda: None
        main = torch.cuda.current_stream(self.dev)
        ss = self.side.side_stream
        ss.wait_stream(main)
        with torch.cuda.stream(ss):
            fn(self.side)
        return lambda: main.wait_stream(ss)

    # ------------------------------------------------------------------ fused GroupNorm statistics
    def _gn_acc(self) -> torch.Tensor:
        i = self._gn_next
        if i >= self._gn_slots:   # a GroupNorm site the arena was not sized for: fail, never hand out past the end
            raise RuntimeError(f"GroupNorm accumulator arena exhausted ({self._gn_slots} slots)")
        self._gn_next += 1
        return self.gn_arena[i * self._gn_words:(i + 1) * self._gn_words]

    def _gn_pays(self, hw, c, backward):
        return self.fuse_gn and bool(ops.call_int("dc_gn_fuse_pays", hw, c, self.groups, int(backward)))

    def _gn_consumer(self, x, c, hw, x2=None, c1=0):
        """A forward GroupNorm over x (channels >= c1 from x2): its accumulator, registered with the producers (None:
        the separate-pass GroupNorm, where fusing does not pay, dc_gn_fuse_pays)."""
        if not self._gn_pays(hw, c, False):
            return None
        acc = self._gn_acc()
        cpg = c // self.groups
        self._gn_targets.setdefault(id(x), []).append((acc, 0, self.groups, cpg, hw))
        if x2 is not None:
            self._gn_targets.setdefault(id(x2), []).append((acc, c1, self.groups, cpg, hw))
        return acc

    def _conv_fwd(self, x, w, y, linear=False, **kw):
        """A forward conv / linear producing y, with the fused GroupNorm statistics of y's consumers (_gnf)."""
        if linear:
            rows, cout = kw.pop("rows"), kw.pop("cout")
            kw = dict(nb=1, hin=1, win=rows, cin=w.shape[1], hout=1, wout=rows, cout=cout, kh=1, kw=1, pad=0, **kw)
        ops.conv_gemm(self.ctx, x, w, y=y, gn=self._gnf(y), **kw)

    def _gnf(self, y):
        """dc_gn_fuse (mode 1) for a conv writing y, or None when no GroupNorm reads y."""
        if not self.fuse_gn:
            return None
        g = self._gn_fuse.get(id(y))
        if g is None:
            tg = self._gn_targets.get(id(y))
            if tg is None:
                return None
            g = self._gn_fuse[id(y)] = ops.gn_fuse_fwd(tg)
        return g

    def _gn_fwd(self, x, hw, c, norm, silu, acc, y, stats, x2=None, c1=0):
        if acc is not None:
            ops.groupnorm_acc(self.ctx, x, self.nb, hw, c, norm.gamma, norm.beta, norm.eps, silu, acc, y, stats,
                              x2=x2, c1=c1, groups=self.groups)
        else:
            ops.groupnorm(self.ctx, x, self.nb, hw, c, norm.gamma, norm.beta, norm.eps, silu, y, stats, x2=x2, c1=c1,
                          groups=self.groups)

    def _gn_bwd_fuse(self, x, hw, c, norm, silu, stats, x2=None, c1=0):
        """(accumulator, dc_gn_fuse mode 2) for the conv producing dL/d(GroupNorm output), or (None, None)."""
        if not self._gn_pays(hw, c, True):
            return None, None
        acc = self._gn_acc()
        return acc, ops.gn_fuse_bwd(acc, self.groups, c // self.groups, hw, x, stats, norm.gamma, norm.beta, silu,
                                    x2=x2, c1=c1)

    def _gn_bwd(self, x, hw, c, norm, silu, stats, acc, dy, dx, x2=None, c1=0, add1=None, add2=None):
        if acc is not None:
            ops.groupnorm_bwd_acc(self.ctx, x, self.nb, hw, c, norm.gamma, stats, acc, dy, dx, x2=x2, c1=c1,
                                  add1=add1, add2=add2, groups=self.groups)
        else:
            ops.groupnorm_bwd(self.ctx, x, self.nb, hw, c, norm.gamma, norm.beta, silu, stats, dy, dx, x2=x2, c1=c1,
                              add1=add1, add2=add2, groups=self.groups)

    # ------------------------------------------------------------------ forward
    def _resnet(self, r: ResnetW, x, hw, x2=None, c1=0):
        ctx, nb = self.ctx, self.nb
        hh, ww = hw
        P = nb * hh * ww
        cin, cout = r.cin, r.cout
        g1 = self.buf(P, cin)
        st1 = self.fbuf(nb, 32, 2)
        h1 = self.buf(P, cout)
        st2 = self.fbuf(nb, 32, 2)
        g2 = self.buf(P, cout)
        out = self.buf(P, cout)
        sc = self.buf(P, cout) if r.shortcut is not None else None
        acc1 = self._gn_consumer(x, cin, hh * ww, x2=x2, c1=c1)
        acc2 = self._gn_consumer(h1, cout, hh * ww)

        def f():
            join = None
            if r.shortcut is not None:
                join = self._branch(lambda c: ops.conv_gemm(
                    c, x, r.shortcut.wf, nb=nb, hin=hh, win=ww, cin=cin, hout=hh, wout=ww, cout=cout, kh=1, kw=1,
                    pad=0, x2=x2, c1=c1, bias=r.shortcut.bias, y=sc))
            self._gn_fwd(x, hh * ww, cin, r.norm1, True, acc1, g1, st1, x2=x2, c1=c1)
            self._conv_fwd(g1, r.conv1.wf, h1, nb=nb, hin=hh, win=ww, cin=cin, hout=hh, wout=ww, cout=cout,
                           bias=r.conv1.bias, rowbias=r.temb_table, rowbias_ld=cout)
            self._gn_fwd(h1, hh * ww, cout, r.norm2, True, acc2, g2, st2)
            res = x
            if join is not None:
                join()
                res = sc
            self._conv_fwd(g2, r.conv2.wf, out, nb=nb, hin=hh, win=ww, cin=cout, hout=hh, wout=ww, cout=cout,
                           bias=r.conv2.bias, resid=res)

        self.fwd.append(f)
        self.tape.append(("resnet", dict(r=r, x=x, x2=x2, c1=c1, hw=hw, st1=st1, h1=h1, st2=st2, out=out)))
        return out

    def _transformer(self, t: TransformerW, x, hw):
        ctx, nb = self.ctx, self.nb
        hh, ww = hw
        T = hh * ww
        P = nb * T
        C, H = t.c, t.heads
        if t.cross_tabs is None:
            t.cross_tabs = ops.crossattn_tables(ctx, t.U, t.D, H, C)
        fused = t.ln_fused
        n0 = self.buf(P, C)
        st0 = self.fbuf(nb, 32, 2)
        p = self.buf(P, C)
        l1 = self.buf(P, C)
        sl1 = self.fbuf(P, 2)
        qkv = self.buf(P, 3 * C)
        o = self.buf(P, C)
        lse = self.fbuf(nb, H, T)
        r1 = self.buf(P, C)
        r2 = self.buf(P, C)
        sl2 = self.fbuf(P, 2)
        probs = self.fbuf(P, H)
        l3 = None if fused else self.buf(P, C)
        sl3 = self.fbuf(P, 2)
        lnf3 = ops.ln_fuse(t.ff1, sl3) if fused else None
        self.saved.append(lnf3)
        f8 = self.buf(P, 8 * C)
        gg = self.buf(P, 4 * C)
        r3 = self.buf(P, C) if t.ffo is None else None
        out = self.buf(P, C)
        acc0 = self._gn_consumer(x, C, T)

        def f():
            self._gn_fwd(x, T, C, t.norm, False, acc0, n0, st0)
            ops.linear(ctx, n0, t.proj_in.wf, P, C, p, bias=t.proj_in.bias)
            ops.layernorm(ctx, p, P, C, t.ln1.gamma, t.ln1.beta, t.ln1.eps, l1, sl1)
            ops.linear(ctx, l1, t.qkv.wf, P, 3 * C, qkv)
            ops.attn_fwd(ctx, qkv, nb, T, H, o, lse)
            ops.linear(ctx, o, t.out.wf, P, C, r1, bias=t.out.bias, resid=p)
            # (fused: with norm3's row statistics of its output r2)
            ops.crossattn_fwd(ctx, r1, P, C, H, t.ln2.eps, t.ln2.gamma, t.ln2.beta, t.cross_tabs, t.c0, r2, sl2,
                              probs, ystats=sl3 if fused else None, yeps=t.ln3.eps)
            if fused:   # norm3 inside ff.net.0.proj (+ GEGLU)
                ops.linear(ctx, r2, t.ff1.wf, P, 8 * C, f8, geglu=1, y2=gg, ln=lnf3)
            else:
                ops.layernorm(ctx, r2, P, C, t.ln3.gamma, t.ln3.beta, t.ln3.eps, l3, sl3)
                ops.linear(ctx, l3, t.ff1.wf, P, 8 * C, f8, bias=t.ff1.bias, geglu=1, y2=gg)   # + GEGLU
            if t.ffo is not None:   # (FF2 + residual) -> proj_out + residual as one linear over [gg | r2]
                self._conv_fwd(gg, t.ffo.wf, out, linear=True, rows=P, cout=C, bias=t.ffo.bias, resid=x, x2=r2,
                               c1=4 * C)
            else:
                ops.linear(ctx, gg, t.ff2.wf, P, C, r3, bias=t.ff2.bias, resid=r2)
                self._conv_fwd(r3, t.proj_out.wf, out, linear=True, rows=P, cout=C, bias=t.proj_out.bias, resid=x)

        self.fwd.append(f)
        self.tape.append(("transformer", dict(t=t, x=x, hw=hw, st0=st0, p=p, sl1=sl1, qkv=qkv, o=o, lse=lse, r1=r1,
                                              r2=r2, sl2=sl2, probs=probs, sl3=sl3, f8=f8, out=out)))
        return out

    def _downsample(self, cv: Conv, x, hw):
        ctx, nb = self.ctx, self.nb
        hh, ww = hw
        ho, wo = _conv_out_hw(hh, 2), _conv_out_hw(ww, 2)
        out = self.buf(nb * ho * wo, cv.cout)

        def f():
            self._conv_fwd(x, cv.wf, out, nb=nb, hin=hh, win=ww, cin=cv.cin, hout=ho, wout=wo, cout=cv.cout, stride=2,
                           bias=cv.bias)

        self.fwd.append(f)
        self.tape.append(("down", dict(cv=cv, x=x, hw=hw, ohw=(ho, wo), out=out)))
        return out, (ho, wo)

    def _upsample(self, cv: Conv, x, hw, ohw):
        ctx, nb = self.ctx, self.nb
        hh, ww = hw
        ho, wo = ohw
        out = self.buf(nb * ho * wo, cv.cout)

        def f():
            self._conv_fwd(x, cv.wf, out, nb=nb, hin=hh, win=ww, cin=cv.cin, hout=ho, wout=wo, cout=cv.cout, mode=1,
                           bias=cv.bias)

        self.fwd.append(f)
        self.tape.append(("up", dict(cv=cv, x=x, hw=hw, ohw=ohw, out=out)))
        return out

    def _build_forward(self):
        net, ctx, nb = self.net, self.ctx, self.nb
        cfg = net.cfg
        hw = (self.h, self.w)
        c0 = cfg.block_out_channels[0]
        h0 = self.buf(nb * self.h * self.w, c0)
        x8 = self.x8

        def f_in():
            if self.fuse_gn:   # every accumulator of the step (forward and backward) starts at zero
                ops.memset(ctx, self.gn_arena)
            ops.conv_gemm(ctx, x8, net.conv_in.wf, nb=nb, hin=self.h, win=self.w, cin=8, hout=self.h, wout=self.w,
                          cout=c0, bias=net.conv_in.bias, y=h0, gn=self._gnf(h0))

        self.fwd.append(f_in)
        self.tape.append(("conv_in", dict(out=h0)))
        skips = [(h0, hw)]
        x = h0
        sizes = [hw]
        for i, blk in enumerate(net.down):
            for j, r in enumerate(blk["resnets"]):
                x = self._resnet(r, x, hw)
                if blk["attns"]:
                    x = self._transformer(blk["attns"][j], x, hw)
                skips.append((x, hw))
            if blk["down"] is not None:
                x, hw = self._downsample(blk["down"], x, hw)
                skips.append((x, hw))
                sizes.append(hw)
        x = self._resnet(net.mid_res[0], x, hw)
        x = self._transformer(net.mid_attn, x, hw)
        x = self._resnet(net.mid_res[1], x, hw)
        for i, blk in enumerate(net.up):
            for j, r in enumerate(blk["resnets"]):
                s, shw = skips.pop()
                assert shw == hw
                c1 = x.shape[1]
                x = self._resnet(r, x, hw, x2=s, c1=c1)
                if blk["attns"]:
                    x = self._transformer(blk["attns"][j], x, hw)
            if blk["up"] is not None:
                ohw = skips[-1][1]  # diffusers forward_upsample_size: upsample to the next skip's size
                x = self._upsample(blk["up"], x, hw, ohw)
                hw = ohw
        # head: GN + SiLU + conv_out
        P = nb * self.h * self.w
        g = self.buf(P, c0)
        st = self.fbuf(nb, 32, 2)
        xin = x
        acc_h = self._gn_consumer(xin, c0, self.h * self.w)

        def f_out():
            self._gn_fwd(xin, self.h * self.w, c0, net.norm_out, True, acc_h, g, st)
            ops.conv_gemm(ctx, g, net.conv_out.wf, nb=nb, hin=self.h, win=self.w, cin=c0, hout=self.h, wout=self.w,
                          cout=4, bias=net.conv_out.bias, y=self.v)

        self.fwd.append(f_out)
        self.tape.append(("head", dict(x=xin, st=st)))

    # ------------------------------------------------------------------ backward
    def _build_backward(self):
        net, ctx, nb = self.net, self.ctx, self.nb
        grad_of = {}   # id(tensor) -> grad tensor / Slice
        extra_of = {}  # id(skip tensor) -> Slice of the up-resnet's concat gradient
        dev_h, dev_w = self.h, self.w
        bwd = []
        for kind, d in reversed(self.tape):
            if kind == "head":
                x = d["x"]
                P = nb * dev_h * dev_w
                c0 = x.shape[1]
                dg = self.buf(P, c0)
                dx = self.buf(P, c0)
                grad_of[id(x)] = dx
                st = d["st"]
                accb, gnb = self._gn_bwd_fuse(x, dev_h * dev_w, c0, net.norm_out, True, st)

                def b(x=x, dg=dg, dx=dx, st=st, c0=c0, accb=accb, gnb=gnb):
                    ops.conv_gemm(ctx, self.dv, net.conv_out.wd, nb=nb, hin=dev_h, win=dev_w, cin=8, hout=dev_h,
                                  wout=dev_w, cout=c0, y=dg, gn=gnb)
                    self._gn_bwd(x, dev_h * dev_w, c0, net.norm_out, True, st, accb, dg, dx)

                bwd.append(b)
            elif kind == "up":
                cv, x, (hh, ww), (ho, wo), out = d["cv"], d["x"], d["hw"], d["ohw"], d["out"]
                dout = grad_of[id(out)]
                dhi = self.buf(nb * ho * wo, cv.cin)
                dx = self.buf(nb * hh * ww, cv.cin)
                grad_of[id(x)] = dx

                def b(cv=cv, dout=dout, dhi=dhi, dx=dx, hh=hh, ww=ww, ho=ho, wo=wo):
                    ops.conv_gemm(ctx, dout, cv.wd, nb=nb, hin=ho, win=wo, cin=cv.cout, hout=ho, wout=wo,
                                  cout=cv.cin, y=dhi)
                    ops.upsample_adjoint(ctx, dhi, nb, ho, wo, cv.cin, hh, ww, dx)

                bwd.append(b)
            elif kind == "down":
                cv, x, (hh, ww), (ho, wo), out = d["cv"], d["x"], d["hw"], d["ohw"], d["out"]
                dout = grad_of[id(out)]
                dx = self.buf(nb * hh * ww, cv.cin)
                grad_of[id(x)] = dx
                extra = extra_of.get(id(x))

                def b(cv=cv, dout=dout, dx=dx, hh=hh, ww=ww, ho=ho, wo=wo, extra=extra):
                    ops.conv_gemm(ctx, dout, cv.wd, nb=nb, hin=ho, win=wo, cin=cv.cout, hout=hh, wout=ww,
                                  cout=cv.cin, mode=2, resid=extra, y=dx)

                bwd.append(b)
            elif kind == "transformer":
                bwd.append(self._transformer_bwd(d, grad_of, extra_of))
            elif kind == "resnet":
                bwd.append(self._resnet_bwd(d, grad_of, extra_of))
            elif kind == "conv_in":
                out = d["out"]
                dout = grad_of[id(out)]

                def b(dout=dout):
                    ops.conv_gemm(ctx, dout, net.conv_in.wd, nb=nb, hin=dev_h, win=dev_w, cin=net.conv_in.cout,
                                  hout=dev_h, wout=dev_w, cout=4, y=self.gx)

                bwd.append(b)
        self.bwd = bwd

    def _resnet_bwd(self, d, grad_of, extra_of):
        ctx, nb = self.ctx, self.nb
        r, x, x2, c1, (hh, ww) = d["r"], d["x"], d["x2"], d["c1"], d["hw"]
        st1, h1, st2, out = d["st1"], d["h1"], d["st2"], d["out"]
        P = nb * hh * ww
        cin, cout = r.cin, r.cout
        dout = grad_of[id(out)]
        dg2 = self.buf(P, cout)
        dh1 = self.buf(P, cout)
        dg1 = self.buf(P, cin)
        dx = self.buf(P, cin)
        if x2 is not None:
            grad_of[id(x)] = Slice(dx, 0)
            extra_of[id(x2)] = Slice(dx, c1)
            extra = None
        else:
            grad_of[id(x)] = dx
            extra = extra_of.get(id(x))

        acc2, gn2 = self._gn_bwd_fuse(h1, hh * ww, cout, r.norm2, True, st2)
        acc1, gn1 = self._gn_bwd_fuse(x, hh * ww, cin, r.norm1, True, st1, x2=x2, c1=c1)
        # the shortcut's input-gradient (a side branch, _branch) lands in its own buffer and enters dx as the
        # GroupNorm backward's first addend, where the identity shortcut's dout goes
        dsc = self.buf(P, cin) if r.shortcut is not None else None

        def b():
            join = None
            if r.shortcut is not None:
                join = self._branch(lambda c: ops.conv_gemm(
                    c, dout, r.shortcut.wd, nb=nb, hin=hh, win=ww, cin=cout, hout=hh, wout=ww, cout=cin, kh=1, kw=1,
                    pad=0, y=dsc))
            ops.conv_gemm(ctx, dout, r.conv2.wd, nb=nb, hin=hh, win=ww, cin=cout, hout=hh, wout=ww, cout=cout, y=dg2,
                          gn=gn2)
            self._gn_bwd(h1, hh * ww, cout, r.norm2, True, st2, acc2, dg2, dh1)
            ops.conv_gemm(ctx, dh1, r.conv1.wd, nb=nb, hin=hh, win=ww, cin=cout, hout=hh, wout=ww, cout=cin, y=dg1,
                          gn=gn1)
            if join is not None:
                join()
            self._gn_bwd(x, hh * ww, cin, r.norm1, True, st1, acc1, dg1, dx, x2=x2, c1=c1,
                         add1=dout if dsc is None else dsc, add2=extra)

        return b

    def _transformer_bwd(self, d, grad_of, extra_of):
        ctx, nb = self.ctx, self.nb
        t, x, (hh, ww) = d["t"], d["x"], d["hw"]
        T = hh * ww
        P = nb * T
        C, H = t.c, t.heads
        out = d["out"]
        dout = grad_of[id(out)]
        dr3 = self.buf(P, C)
        df = self.buf(P, 8 * C)
        dl3 = self.buf(P, C)
        fused = t.ln_fused
        dr2 = None if fused else self.buf(P, C)
        dr1 = self.buf(P, C)
        do = self.buf(P, C)
        dqkv = self.buf(P, 3 * C)
        dl1 = self.buf(P, C)
        dp = self.buf(P, C)
        dn0 = self.buf(P, C)
        dx = self.buf(P, C)
        delta = self.fbuf(2, nb, H, T)   # the backward's row constants: -delta, -8 lse
        grad_of[id(x)] = dx
        extra = extra_of.get(id(x))
        st0, p, sl1, qkv, o, lse = d["st0"], d["p"], d["sl1"], d["qkv"], d["o"], d["lse"]
        r1, r2, sl2, probs, sl3, f8 = d["r1"], d["r2"], d["sl2"], d["probs"], d["sl3"], d["f8"]

        acc0, gn0 = self._gn_bwd_fuse(x, T, C, t.norm, False, st0)

        def b():
            if t.ffo is not None:   # dL/dgg (+ GEGLU backward) and dL/dr2 from one linear
                ops.linear(ctx, dout, t.ffo.wd, P, 5 * C, df, geglu=2, aux=f8, y2=dr3, geglu_n=4 * C)
            else:
                ops.linear(ctx, dout, t.proj_out.wd, P, C, dr3)
                ops.linear(ctx, dr3, t.ff2.wd, P, 4 * C, df, geglu=2, aux=f8)   # + GEGLU backward
            ops.linear(ctx, df, t.ff1.wd, P, C, dl3)   # (fused: gamma3 * dL/dLN3 through the folded weight)
            if fused:   # norm3 backward inside the cross-attention backward
                ops.crossattn_bwd_ln(ctx, r1, P, C, H, t.ln2.gamma, t.cross_tabs, sl2, probs, dl3, r2, sl3, dr3, dr1)
            else:
                ops.layernorm_bwd(ctx, r2, P, C, t.ln3.gamma, sl3, dl3, dr2, add=dr3)
                ops.crossattn_bwd(ctx, r1, P, C, H, t.ln2.gamma, t.cross_tabs, sl2, probs, dr2, dr1)
            ops.linear(ctx, dr1, t.out.wd, P, C, do)
            ops.attn_bwd(ctx, qkv, o, do, lse, nb, T, H, delta, dqkv)
            ops.linear(ctx, dqkv, t.qkv.wd, P, C, dl1)
            ops.layernorm_bwd(ctx, p, P, C, t.ln1.gamma, sl1, dl1, dp, add=dr1)
            ops.linear(ctx, dp, t.proj_in.wd, P, C, dn0, gn=gn0)
            self._gn_bwd(x, T, C, t.norm, False, st0, acc0, dn0, dx, add1=dout, add2=extra)

        return b

    # ------------------------------------------------------------------ run
    def forward(self):
        for f in self.fwd:
            f()
        return self.v

    def backward(self):
        for b in self.bwd:
            b()
        return self.gx

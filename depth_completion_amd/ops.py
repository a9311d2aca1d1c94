"""Thin host wrappers: torch device tensors -> raw pointers -> libdcamd.so entry points.

Tensors are 2-D "row" views ``[rows, ld]`` (NHWC pixel rows or token rows).  ``Slice`` carries
a column offset into a row buffer (for concat halves and q/k/v blocks) without copying.
PyTorch is used only for device memory and the current stream handle.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
from dataclasses import dataclass
from pathlib import Path

import torch

from . import _lib
from ._lib import ConvDesc, GnFuse, LnFuse, call

BF16 = torch.bfloat16


@dataclass
class Slice:
    t: torch.Tensor
    col: int = 0

    @property
    def ld(self) -> int:
        return self.t.shape[-1]

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + self.col * self.t.element_size()


def S(t, col: int = 0) -> Slice:
    return t if isinstance(t, Slice) else Slice(t, col)


def P(t) -> int | None:
    """Raw device pointer of a tensor / Slice / None."""
    if t is None:
        return None
    if isinstance(t, Slice):
        return t.ptr
    return t.data_ptr()


def LD(t) -> int:
    if t is None:
        return 0
    return t.ld if isinstance(t, Slice) else t.shape[-1]


TUNED_TABLE = Path(os.environ.get("DC_TUNED") or Path(__file__).resolve().parent / "tuned_gfx950.json")


def load_tuned(path: Path = TUNED_TABLE) -> dict:
    """Committed (algo, splitk) choices per conv shape, measured on MI355X by tools/tune_gemm.py."""
    if not path.exists():
        return {}
    return {tuple(e["key"]): (e["algo"], e["splitk"]) for e in json.loads(path.read_text())}


def save_tuned(cache: dict, path) -> None:
    ent = [{"key": list(k), "algo": a, "splitk": s} for k, (a, s) in sorted(cache.items())]
    Path(path).write_text(json.dumps(ent, indent=0))


class Ctx:
    """Execution context: stream, fp32 scratch workspace and the device step counter.

    ``algo_cache`` maps a conv shape key to the (tile algo, split-K) variant of dc_conv_gemm; it
    starts from the committed tuned table.  With ``tune`` (env DC_TUNE=1) a shape missing from
    the cache is timed over every variant on the call's own operands the first time it runs
    eagerly (never while a hipGraph is being captured); otherwise the library heuristic runs.
    """

    def __init__(self, device, ws_mb: int = 96, tune: bool | None = None):
        self.device = torch.device(device)
        # zero-filled: the split-K tile counters at its end must start at 0 (dc_conv_gemm keeps them so)
        self.ws = torch.zeros(ws_mb * (1 << 20) // 4, dtype=torch.float32, device=self.device)
        self.step = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.algo_cache: dict = load_tuned()
        self.tune = os.environ.get("DC_TUNE") == "1" if tune is None else tune
        # the committed table in file order, for dc_conv_pick's nearest-shape choice (the native session passes
        # the same table in the same order, so both hosts launch the same variants)
        self._table = list(self.algo_cache.items())
        self._picked: dict = {}

    def choose_algo(self, d, y=None, srcs=()):
        """(algo, splitk) for a conv descriptor: tuned table / autotune; a shape missing from the table takes
        the variant of the nearest tuned shape (dc_conv_pick; DC_GEMM_NN=0: the library heuristic instead)."""
        key = conv_key(d)
        if key not in self.algo_cache and self.tune and self.device.type == "cuda" \
                and not torch.cuda.is_current_stream_capturing():
            self.algo_cache[key] = _autotune(self, d, y, srcs=srcs)
        if key in self.algo_cache:
            return self.algo_cache[key]
        if key not in self._picked:
            self._picked[key] = pick_variant(self._table, key)
        return self._picked[key]

    def side(self) -> "Ctx":
        """A context for a concurrent graph branch: its own stream (``side_stream``) and its own workspace (split-K
        partials and tile counters must not be shared with the main stream's launches), the same variant tables."""
        s = self.__dict__.get("_side")
        if s is None:
            s = object.__new__(Ctx)
            s.__dict__.update(self.__dict__)
            s.ws = torch.zeros_like(self.ws)
            s.side_stream = torch.cuda.Stream(self.device)
            self._side = s
        return s

    @property
    def stream(self) -> int:
        if self.device.type != "cuda":
            return 0  # host-side dry runs (tests/test_host_plans.py) only
        return torch.cuda.current_stream(self.device).cuda_stream

    @property
    def ws_bytes(self) -> int:
        return self.ws.numel() * 4


# ------------------------------------------------------------------------- conv / linear
def conv_key(d) -> tuple:
    return (d.mode, d.nb, d.hin, d.win, d.cin, d.hout, d.wout, d.cout, d.kh, d.stride, bool(d.x2), d.ktot)


def pick_variant(table: list, key: tuple) -> tuple:
    """dc_conv_pick over ``table`` [(key, (algo, splitk))] in order: exact match, else the nearest tuned shape."""
    if not table or os.environ.get("DC_GEMM_NN") == "0":
        return (0, 0)
    keys = (C.c_int * (12 * len(table)))(*[int(v) for k, _ in table for v in k])
    choices = (C.c_int * (2 * len(table)))(*[int(v) for _, c in table for v in c])
    kk = (C.c_int * 12)(*[int(v) for v in key])
    out = (C.c_int * 2)()
    _lib.load().dc_conv_pick(C.addressof(keys), C.addressof(choices), len(table), C.addressof(kk), C.addressof(out))
    return (out[0], out[1])


def conv_gemm(ctx: Ctx, x, w: torch.Tensor, *, y=None, **kw):
    """rows: optional (int32 tensor, count) -- compute only those output pixels (sorted row indices)."""
    d = conv_desc(ctx, x, w, y=y, **kw)
    call("dc_conv_gemm", C.byref(d), ctx.stream)
    return y


def conv_desc(ctx: Ctx, x, w: torch.Tensor, *, nb: int, hin: int, win: int, cin: int, hout: int, wout: int,
              cout: int, kh: int = 3, kw: int = 3, stride: int = 1, pad: int = 1, mode: int = 0, x2=None,
              c1: int = 0, bias=None, rowbias=None, rowbias_ld: int = 0, resid=None, mask=None, act: int = 0,
              y=None, splitk: bool = True, algo: int | None = None, nsplit: int | None = None, geglu: int = 0,
              y2=None, aux=None, rows=None, gn: GnFuse | None = None, ln: LnFuse | None = None, geglu_n: int = 0):
    """The dc_conv_desc of one conv_gemm call, its (algo, split) chosen (tuned table / nearest shape).
    gn: fused GroupNorm statistics (include/dcamd.h dc_gn_fuse; the caller keeps it alive); ln: a LayerNorm of the
    input rows folded in (dc_ln_fuse, ln_fuse below; the caller keeps it alive)."""
    d = ConvDesc()
    d.x = P(x)
    d.ldx = LD(x)
    d.x2 = P(x2)
    d.ldx2 = LD(x2)
    d.c1 = c1
    d.nb, d.hin, d.win, d.cin, d.hout, d.wout = nb, hin, win, cin, hout, wout
    d.kh, d.kw, d.stride, d.pad, d.mode = kh, kw, stride, pad, mode
    d.w = w.data_ptr()
    d.ktot = w.shape[1]
    d.cout = cout
    d.bias = P(bias)
    d.rowbias = P(rowbias)
    d.rowbias_idx = ctx.step.data_ptr() if rowbias is not None else None
    d.rowbias_ld = rowbias_ld
    d.resid = P(resid)
    d.ldr = LD(resid)
    d.mask = P(mask)
    d.ldmask = LD(mask)
    d.act = act
    d.y = P(y)
    d.ldy = LD(y)
    d.geglu = geglu
    d.y2 = P(y2)
    d.ldy2 = LD(y2)
    d.aux = P(aux)
    d.ldaux = LD(aux)
    d.geglu_n = geglu_n
    d.ws = ctx.ws.data_ptr() if splitk else None
    d.ws_bytes = ctx.ws_bytes if splitk else 0
    if gn is not None:
        d.gn = C.pointer(gn)
    if ln is not None:
        d.ln = C.pointer(ln)
    if rows is not None:
        d.rows, d.nrows = rows[0].data_ptr(), int(rows[1])
        if algo is None:   # row counts vary per call: the library heuristic on nrows, not the tuned table
            algo, nsplit = 0, 0
    if algo is None:
        algo, nsplit = ctx.choose_algo(d, y, srcs=(x, x2, resid))
    d.algo = algo
    d.splitk = nsplit or 0
    return d


HALO_FIRST, HALO_LAST = 23, 36   # dc_conv_gemm algo ids of the halo-tile direct 3x3 conv (conv_gemm_impl.h); ids
# 1 .. 22 and 37 .. 42 are im2col tile variants, SKINNY_FIRST .. dc_conv_num_algos() the weight-streaming skinny
# conv / linear variants (conv_skinny.h)
HALOX_FIRST, HALOX_LAST = 62, 66   # the round-4 halo variants (192-px tiles, one block per CU, 8-deep weight ring)
IM2COL_LAST, SKINNY_FIRST, RESIDENT_FIRST, WIDE_FIRST, WIDE_LAST = 42, 43, 55, 59, 61   # RESIDENT_FIRST ..: the weight-resident
# persistent narrow convs (cin 64, cout <= 64; their split field is the persistent grid's blocks per CU); WIDE_FIRST ..
# dc_conv_num_algos(): im2col tiles holding 320 output channels per block
SKINNY_TAPS = (9, 9, 9, 9, 9, 1, 1, 1, 1, 1, 1, 1)   # taps of skinny variant SKINNY_FIRST + i (conv_skinny.h kSkinnyAlgos)


def halo_eligible(d) -> bool:
    """The halo kernel's contract (conv_gemm.hip halo_eligible): 3x3, stride 1, pad 1, direct or nearest-upsample
    input, whole 64-channel chunks, no row list, no GEGLU epilogue."""
    return (d.kh == 3 and d.kw == 3 and d.stride == 1 and d.pad == 1 and d.cin % 64 == 0 and not d.rows
            and not d.geglu and d.mode in (0, 1) and d.ktot == 9 * d.cin
            and (d.mode == 1 or (d.hin == d.hout and d.win == d.wout))
            and (not d.x2 or d.c1 % 64 == 0))


def skinny_eligible(d) -> bool:
    """Shapes the weight-streaming skinny variants serve (conv_skinny.h skinny_eligible, before the per-variant
    chunk-group condition): the halo contract, or a 1x1 / linear over whole 64-channel chunks.  The 1x1 forms are
    tuned only for the few-pixel layers (at most 512 output pixels: UNet levels 2-3 at batch 1); the 3x3 forms at
    every size (the weight-in-VGPR ring with one barrier per chunk group beats the per-tap-barrier halo tiles on the
    level-0 / level-1 convs, profiles/r05af/).  Both carry the fused-GroupNorm-statistics epilogue (conv_skinny.h
    GnTileSums), so a shape's choice serves its fused and unfused calls alike."""
    if d.kh == 1 and d.kw == 1:
        return (d.nb * d.hout * d.wout <= 512 and d.stride == 1 and d.pad == 0 and d.mode == 0 and d.cin % 64 == 0
                and d.ktot == d.cin and not d.rows and not d.geglu and d.hin == d.hout and d.win == d.wout
                and (not d.x2 or d.c1 % 64 == 0))
    return halo_eligible(d)


def _autotune(ctx: Ctx, d, y, reps: int = 3, srcs=()) -> tuple:
    """Time every (algo, splitk) variant of one conv on its own operands; returns the fastest.

    Candidates write a scratch copy of the output so in-place epilogues (resid == y) stay intact.
    DC_TUNE_COLD=1 flushes L2 and the Infinity Cache before every timed call; DC_TUNE_COLD=2 flushes and then
    reads the activation operands back (``srcs``), the cache state of the sampler step, where the input was
    just written by the previous kernel and only the weights are cold.
    """
    rows = d.nb * d.hout * d.wout
    tmp = torch.empty(rows, d.ldy, dtype=BF16, device=ctx.device)
    base = y.t.data_ptr() if isinstance(y, Slice) else y.data_ptr()
    dt = ConvDesc.from_buffer_copy(d)
    dt.y = tmp.data_ptr() + (d.y - base)
    dt.gn = None   # candidates must not add to the GroupNorm accumulators
    nalg = _lib.load().dc_conv_num_algos()
    # im2col tiles: split-K 1..32, and stream-K over 256 / 512 / 768 blocks (splitk -1 / -2 / -3); halo tiles
    # (algos > HALO_FIRST - 1, stride-1 3x3 convs over whole 64-channel chunks only): input-chunk splits
    gemm_ids = list(range(1, HALO_FIRST)) + list(range(HALO_LAST + 1, IM2COL_LAST + 1)) + list(range(WIDE_FIRST, WIDE_LAST + 1))
    cands = [(0, 0)] + [(a, s) for a in gemm_ids for s in (1, 2, 4, 8, 12, 16, 24, 32, -1, -2, -3)]
    if halo_eligible(d):
        cands += [(a, s) for a in list(range(HALO_FIRST, HALO_LAST + 1)) + list(range(HALOX_FIRST, HALOX_LAST + 1))
                  for s in (1, 2, 3, 4, 5, 8, 10, 16, 20) if s <= d.cin // 64]
    if skinny_eligible(d):
        # skinny variants (an ineligible variant reports an error or falls back; both are timed like the rest)
        taps = d.kh * d.kw
        # (splitk < 0: the same split with the partials summed by a second kernel instead of the last-arriving block)
        cands += [(a, s) for a in range(SKINNY_FIRST, RESIDENT_FIRST)
                  for s in (1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, -2, -4, -6, -8, -10, -12, -16, -20)
                  if abs(s) <= d.cin // 64 and SKINNY_TAPS[a - SKINNY_FIRST] == taps]
    if halo_eligible(d) and d.cin == 64 and d.cout <= 64 and not d.gn and not d.x2:
        cands += [(a, b) for a in range(RESIDENT_FIRST, WIDE_FIRST) for b in (0, 1, 2, 3)]
    if d.gn:
        # a GroupNorm-fused call runs resident / wide choices as the library heuristic (those kernels have no
        # fused-statistics epilogue): never offer them, so the table only holds configurations that were timed
        cands = [c for c in cands if not RESIDENT_FIRST <= c[0] <= WIDE_LAST]
    if d.geglu_n:
        # the folded FF2 / proj_out input-gradient runs wide (320-column) choices as the 64 x 64 tile (a wide tile can
        # straddle geglu_n, where the epilogue switches from the GEGLU backward to plain stores): never offer them
        cands = [c for c in cands if not WIDE_FIRST <= c[0] <= WIDE_LAST]
    if d.ln:
        # a LayerNorm-folded linear (dc_conv_gemm's ln branch) runs on the im2col tiles only: any other choice would be
        # replaced by the library heuristic, so the table would store an id whose timing was the heuristic's
        cands = [c for c in cands if c == (0, 0) or 1 <= c[0] <= IM2COL_LAST and not HALO_FIRST <= c[0] <= HALO_LAST]
    if getattr(ctx, "tune_only", None):   # tools/tune_gemm.py --try: the committed choice against these algos only
        cur = ctx.tune_only[1].get(conv_key(d))
        cands = ([cur] if cur else []) + [c for c in cands if c[0] in ctx.tune_only[0]]
    best, best_t = (0, 0), float("inf")
    # DC_TUNE_COLD=1: every timed call starts with L2 and the Infinity Cache flushed (a 512 MiB write),
    # as the weights are in the sampler step (each is touched once per pass)
    cold = os.environ.get("DC_TUNE_COLD") in ("1", "2")
    warm_srcs = [a.t if isinstance(a, Slice) else a for a in srcs if a is not None] \
        if os.environ.get("DC_TUNE_COLD") == "2" else []
    if cold and getattr(ctx, "_flush", None) is None:
        ctx._flush = torch.empty(512 << 20, dtype=torch.uint8, device=ctx.device)
        ctx._sink = torch.empty((), dtype=torch.float32, device=ctx.device)
    timed = []
    for a, s in cands:
        dt.algo, dt.splitk = a, s
        try:
            call("dc_conv_gemm", C.byref(dt), ctx.stream)
        except _lib.DCError:
            continue
        if cold:
            t = 0.0
            for _ in range(reps):
                ctx._flush.fill_(1)
                for src in warm_srcs:
                    torch.sum(src.reshape(-1), dim=0, dtype=torch.float32, out=ctx._sink)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                call("dc_conv_gemm", C.byref(dt), ctx.stream)
                e1.record()
                e1.synchronize()
                t += e0.elapsed_time(e1)
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call("dc_conv_gemm", C.byref(dt), ctx.stream)
            e1.record()
            e1.synchronize()
            t = e0.elapsed_time(e1)
        if t < best_t * 0.97:  # prefer the earlier (heuristic / fewer splits) on near-ties
            best, best_t = (a, s), t
        timed.append((t / reps * 1e3, a, s))
    if getattr(ctx, "tune_top", None) is not None:   # tools/tune_gemm.py --top-out: the runners-up, fastest first
        ctx.tune_top[conv_key(d)] = [(a, s, round(us, 2)) for us, a, s in sorted(timed)[:6]]
    print(f"tuned {conv_key(d)} -> {best} ({best_t / reps * 1e3:.1f} us)", file=sys.stderr,
          flush=True)
    return best


def linear(ctx: Ctx, x, w: torch.Tensor, rows: int, cout: int, y, bias=None, resid=None, rowbias=None,
           rowbias_ld: int = 0, act: int = 0, geglu: int = 0, y2=None, aux=None, algo: int | None = None,
           nsplit: int | None = None, gn: GnFuse | None = None, ln: LnFuse | None = None, geglu_n: int = 0):
    """y[rows, cout] = x[rows, K] @ w[cout, K]^T (+ bias, + resid); geglu 1 / 2: the fused GEGLU
    epilogues of include/dcamd.h (y2 = h * gelu(gate); aux = interleaved pre-activation); ln: LayerNorm(x) as the
    input (w the folded weight, dc_ln_fuse)."""
    return conv_gemm(ctx, x, w, nb=1, hin=1, win=rows, cin=w.shape[1], hout=1, wout=rows, cout=cout, kh=1, kw=1,
                     stride=1, pad=0, bias=bias, resid=resid, rowbias=rowbias, rowbias_ld=rowbias_ld, act=act, y=y,
                     geglu=geglu, y2=y2, aux=aux, algo=algo, nsplit=nsplit, gn=gn, ln=ln, geglu_n=geglu_n)


def ln_fuse(lin, stats) -> LnFuse:
    """dc_ln_fuse of a weights.LnLinear with the input rows' (mean, rstd) in stats [rows][2] fp32."""
    f = LnFuse()
    f.csum, f.cbias, f.stats = lin.csum.data_ptr(), lin.cbias.data_ptr(), stats.data_ptr()
    return f


# ------------------------------------------------------------------------- norms
def groupnorm(ctx: Ctx, x, nb, hw, c, gamma, beta, eps, silu, y, stats, x2=None, c1=0, groups=32):
    call("dc_groupnorm_fwd", P(x), LD(x), P(x2), LD(x2), c1, nb, hw, c, groups, eps, gamma.data_ptr(),
         beta.data_ptr(), int(silu), P(y), LD(y), stats.data_ptr(), ctx.ws.data_ptr(), ctx.stream)
    return y


def groupnorm_bwd(ctx: Ctx, x, nb, hw, c, gamma, beta, silu, stats, dy, dx, x2=None, c1=0, add1=None, add2=None,
                  groups=32):
    call("dc_groupnorm_bwd", P(x), LD(x), P(x2), LD(x2), c1, nb, hw, c, groups, gamma.data_ptr(), beta.data_ptr(),
         int(silu), stats.data_ptr(), P(dy), LD(dy), P(dx), LD(dx), P(add1), LD(add1), P(add2), LD(add2),
         ctx.ws.data_ptr(), ctx.stream)
    return dx


def call_int(name: str, *args) -> int:
    """A libdcamd query that returns a value rather than a status."""
    return int(getattr(_lib.load(), name)(*args))


def gn_acc_words(nb: int, groups: int = 32) -> int:
    """int64 words of one fused-statistics accumulator (dc_gn_acc_bytes: replicas x frames x groups x 2 x 9)."""
    return int(_lib.load().dc_gn_acc_bytes(nb, groups)) // 8


def gn_fuse_fwd(targets) -> GnFuse:
    """dc_gn_fuse mode 1 for an output feeding the GroupNorms ``targets`` [(acc, coff, groups, cpg, hw)]."""
    g = GnFuse()
    g.mode, g.nt = 1, len(targets)
    for k, (acc, coff, groups, cpg, hw) in enumerate(targets):
        g.t[k].acc, g.t[k].coff, g.t[k].groups, g.t[k].cpg, g.t[k].hw = acc.data_ptr(), coff, groups, cpg, hw
    return g


def gn_fuse_bwd(acc, groups, cpg, hw, x, stats, gamma, beta, silu, x2=None, c1=0) -> GnFuse:
    """dc_gn_fuse mode 2: the output is dL/d(GroupNorm(x)(+SiLU)); the epilogue stores dy' and sums into acc."""
    g = GnFuse()
    g.mode, g.nt = 2, 1
    g.t[0].acc, g.t[0].coff, g.t[0].groups, g.t[0].cpg, g.t[0].hw = acc.data_ptr(), 0, groups, cpg, hw
    g.x, g.ldx, g.x2, g.ldx2, g.c1 = P(x), LD(x), P(x2), LD(x2), c1
    g.stats, g.gamma, g.beta, g.silu = stats.data_ptr(), gamma.data_ptr(), beta.data_ptr(), int(silu)
    return g


def groupnorm_acc(ctx: Ctx, x, nb, hw, c, gamma, beta, eps, silu, acc, y, stats, x2=None, c1=0, groups=32):
    """One-pass GroupNorm(+SiLU) from the statistics its producers accumulated (dc_groupnorm_fwd_acc)."""
    call("dc_groupnorm_fwd_acc", P(x), LD(x), P(x2), LD(x2), c1, nb, hw, c, groups, eps, gamma.data_ptr(),
         beta.data_ptr(), int(silu), acc.data_ptr(), P(y), LD(y), stats.data_ptr(), ctx.stream)
    return y


def groupnorm_bwd_acc(ctx: Ctx, x, nb, hw, c, gamma, stats, acc, dyp, dx, x2=None, c1=0, add1=None, add2=None,
                      groups=32):
    """GroupNorm input-gradient from the producer's dy' and accumulated sums (dc_groupnorm_bwd_acc)."""
    call("dc_groupnorm_bwd_acc", P(x), LD(x), P(x2), LD(x2), c1, nb, hw, c, groups, gamma.data_ptr(),
         stats.data_ptr(), acc.data_ptr(), P(dyp), LD(dyp), P(dx), LD(dx), P(add1), LD(add1), P(add2), LD(add2),
         ctx.stream)
    return dx


def layernorm(ctx: Ctx, x, rows, c, gamma, beta, eps, y, stats):
    call("dc_layernorm_fwd", P(x), LD(x), rows, c, eps, gamma.data_ptr(), beta.data_ptr(), P(y), LD(y),
         stats.data_ptr(), ctx.stream)
    return y


def layernorm_bwd(ctx: Ctx, x, rows, c, gamma, stats, dy, dx, add=None):
    """gamma None: dy is gamma * dL/dy already (the input-gradient of a folded weight, dc_ln_fuse)."""
    call("dc_layernorm_bwd", P(x), LD(x), rows, c, P(gamma), stats.data_ptr(), P(dy), LD(dy), P(dx), LD(dx),
         P(add), LD(add), ctx.stream)
    return dx


# ------------------------------------------------------------------------- attention
def attn_fwd(ctx: Ctx, qkv, nb, t, heads, o, lse):
    call("dc_attn_fwd", P(qkv), LD(qkv), nb, t, heads, P(o), LD(o), lse.data_ptr(), ctx.ws.data_ptr(), ctx.ws_bytes,
         ctx.stream)
    return o


def attn_bwd(ctx: Ctx, qkv, o, dout, lse, nb, t, heads, delta, dqkv):
    if delta.numel() < 2 * nb * heads * t:   # ABI 21: -delta and -8 lse, the dK/dV kernel's row constants
        raise ValueError(f"attn_bwd: delta workspace holds {delta.numel()} floats, needs 2 * nb * heads * t")
    call("dc_attn_bwd", P(qkv), LD(qkv), P(o), LD(o), P(dout), LD(dout), lse.data_ptr(), nb, t, heads,
         delta.data_ptr(), P(dqkv), LD(dqkv), ctx.ws.data_ptr(), ctx.ws_bytes, ctx.stream)
    return dqkv


def crossattn_tables(ctx: Ctx, U, D, heads, c) -> torch.Tensor:
    """bf16 hi / lo MFMA operand tables of the folded cross-attention (dc_crossattn_prepare), once at load."""
    nbytes = _lib.load().dc_crossattn_tables_bytes(heads, c)
    tabs = torch.empty(nbytes // 2, dtype=BF16, device=ctx.device)
    call("dc_crossattn_prepare", U.data_ptr(), D.data_ptr(), heads, c, tabs.data_ptr(), ctx.stream)
    return tabs


def crossattn_fwd(ctx: Ctx, x, rows, c, heads, eps, gamma, beta, tabs, c0, y, stats, probs, ystats=None,
                  yeps=1e-5):
    """ystats: [rows][2] (mean, rstd with yeps) of the output rows (norm3's statistics for dc_ln_fuse), or None."""
    call("dc_crossattn_fwd", P(x), LD(x), rows, c, heads, eps, gamma.data_ptr(), beta.data_ptr(), tabs.data_ptr(),
         c0.data_ptr(), P(y), LD(y), stats.data_ptr(), probs.data_ptr(), P(ystats), yeps, ctx.stream)
    return y


def crossattn_bwd_ln(ctx: Ctx, x, rows, c, heads, gamma, tabs, stats, probs, dl, x3, stats3, add, dx):
    """crossattn_bwd whose dy = LayerNorm3 backward of dl (gamma folded in, dc_ln_fuse) over x3, plus add, computed
    in the same launch (dc_crossattn_bwd_ln)."""
    call("dc_crossattn_bwd_ln", P(x), LD(x), rows, c, heads, gamma.data_ptr(), tabs.data_ptr(), stats.data_ptr(),
         probs.data_ptr(), P(dl), LD(dl), P(x3), LD(x3), stats3.data_ptr(), P(add), LD(add), P(dx), LD(dx),
         ctx.stream)
    return dx


def crossattn_bwd(ctx: Ctx, x, rows, c, heads, gamma, tabs, stats, probs, dy, dx):
    call("dc_crossattn_bwd", P(x), LD(x), rows, c, heads, gamma.data_ptr(), tabs.data_ptr(), stats.data_ptr(),
         probs.data_ptr(), P(dy), LD(dy), P(dx), LD(dx), ctx.stream)
    return dx


# ------------------------------------------------------------------------- elementwise
def geglu(ctx: Ctx, f, rows, c, y):
    call("dc_geglu_fwd", P(f), LD(f), rows, c, P(y), LD(y), ctx.stream)
    return y


def geglu_bwd(ctx: Ctx, f, rows, c, dy, df):
    call("dc_geglu_bwd", P(f), LD(f), rows, c, P(dy), LD(dy), P(df), LD(df), ctx.stream)
    return df


def upsample_adjoint(ctx: Ctx, dhi, nb, hhi, whi, c, hlo, wlo, dlo, mask=None):
    call("dc_upsample_adjoint", P(dhi), LD(dhi), nb, hhi, whi, c, hlo, wlo, P(dlo), LD(dlo), P(mask), LD(mask),
         ctx.stream)
    return dlo


def silu(ctx: Ctx, x, y):
    call("dc_silu", P(x), x.numel(), P(y), ctx.stream)
    return y


def memset(ctx: Ctx, t: torch.Tensor, value: int = 0):
    call("dc_memset_async", t.data_ptr(), value, t.numel() * t.element_size(), ctx.stream)

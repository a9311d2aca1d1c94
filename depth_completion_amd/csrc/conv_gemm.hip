// C ABI of the implicit-GEMM conv / linear (dc_conv_gemm): argument checks, variant choice and launch.  The kernels
// are in conv_gemm_impl.h; the fused GroupNorm-statistics instantiations are compiled in conv_gemm_gn.hip / conv_gemm_gnb.hip.
#include "conv_gemm_impl.h"

namespace {
#include "conv_skinny.h"
}  // namespace
int conv_launch_skinny9(int i, ConvGemmParams& p, int splits, hipStream_t s);
int conv_launch_skinny1(int i, ConvGemmParams& p, int splits, hipStream_t s);
int conv_launch_resident(int i, ConvGemmParams& p, int bpc, hipStream_t s);

// external algo ids: 1 .. kNumAll im2col / halo variants (conv_gemm_impl.h), then the weight-streaming skinny variants,
// then the weight-resident persistent narrow convs (conv_skinny.h), then the wide im2col tiles (conv_gemm_impl.h)
static_assert(kNumAll + kNumSkinny + kNumResident + 1 == kWideFirst, "external algo id blocks");
constexpr int kNumExt = kHaloXFirst + kNumHaloX - 1;
extern "C" int dc_conv_num_algos(void) { return kNumExt; }

// the kernel parameters of a descriptor, checked (DC_OK or the error status); M = output rows
static int conv_params(const dc_conv_desc* d, ConvGemmParams& p, long& M_out) {
  if (!d || !d->x || !d->w || !d->y) return DC_ERR_ARG;
  p.x = (const bf16*)d->x;
  p.x2 = (const bf16*)(d->x2 ? d->x2 : d->x);
  p.ldx = d->ldx;
  p.ldx2 = d->x2 ? d->ldx2 : d->ldx;
  p.c1 = d->x2 ? d->c1 : (1 << 30);
  p.nb = d->nb; p.hin = d->hin; p.win = d->win; p.cin = d->cin;
  p.hout = d->hout; p.wout = d->wout;
  p.kh = d->kh; p.kw = d->kw; p.stride = d->stride; p.pad = d->pad; p.mode = d->mode;
  p.w = (const bf16*)d->w; p.ktot = d->ktot; p.cout = d->cout;
  p.bias = d->bias;
  p.rowbias = (const bf16*)d->rowbias; p.rowbias_idx = d->rowbias_idx; p.rowbias_ld = d->rowbias_ld;
  p.resid = (const bf16*)d->resid; p.ldr = d->ldr;
  p.mask = (const bf16*)d->mask; p.ldmask = d->ldmask;
  p.act = d->act;
  p.y = (bf16*)d->y; p.ldy = d->ldy;
  p.ws = d->ws;
  p.ws_bytes = d->ws_bytes < (1L << 31) ? d->ws_bytes : (1L << 31);  // 32-bit buffer offsets
  p.splits = 1; p.kps = 0; p.counters = nullptr; p.sk_blocks = 0;
  p.geglu = d->geglu;
  p.geglu_n = d->geglu_n;
  p.y2 = (bf16*)d->y2; p.ldy2 = d->ldy2;
  p.aux = (const bf16*)d->aux; p.ldaux = d->ldaux;
  p.rows = d->rows; p.nrows = d->rows ? d->nrows : 0;
  // tile order: M-major (split-major for split-K).  N-major -- (column tile, split, row tile), each XCD's range
  // sharing W slices -- measured no better on the weight-heavy level-2 / 3 shapes and 1.5x slower at batch 8
  // (profiles/r02f/gemm_order_ab.txt); kept opt-in for experiments (DC_GEMM_ORDER=2)
  {
    const char* e = getenv("DC_GEMM_ORDER");
    p.nmajor = (e && atoi(e) == 2) ? 1 : 0;
    const char* dg = getenv("DC_HALO_DIAG");
    p.diag = dg ? atoi(dg) : 0;
  }
  if (p.geglu < 0 || p.geglu > 2) return DC_ERR_ARG;
  if (p.rows && (p.nrows <= 0 || p.geglu)) return DC_ERR_ARG;
  if (p.geglu) {  // plain linear / conv output only: no residual, mask, row bias or activation
    if (p.resid || p.mask || p.rowbias || p.act || p.cout % 16) return DC_ERR_ARG;
    if (p.geglu == 1 && (!p.y2 || p.ldy2 % 8 || ((uintptr_t)p.y2 & 15))) return DC_ERR_ARG;
    const int gn_cols = (p.geglu == 2 && p.geglu_n) ? p.geglu_n : p.cout;   // the GEGLU-backward columns
    if (p.geglu == 2 && (!p.aux || p.ldaux % 8 || ((uintptr_t)p.aux & 15) || p.ldy < 2 * gn_cols)) return DC_ERR_ARG;
    if (p.geglu_n && (p.geglu != 2 || p.geglu_n < 0 || p.geglu_n >= p.cout || p.geglu_n % 256 || !p.y2 ||
                      p.ldy2 % 8 || ((uintptr_t)p.y2 & 15) || p.ldy2 < p.cout - p.geglu_n))
      return DC_ERR_ARG;
  } else if (p.geglu_n) {
    return DC_ERR_ARG;
  }
  // shape / alignment contract (host pads channels, see DESIGN.md "layouts")
  if (p.ktot % 64 != 0 || p.ktot < p.kh * p.kw * p.cin) return DC_ERR_ARG;
  if (p.cin % 8 != 0 || p.cout <= 0 || p.nb <= 0 || p.hout <= 0 || p.wout <= 0) return DC_ERR_ARG;
  if (p.rowbias && !p.rowbias_idx) return DC_ERR_ARG;
  if (p.mode < 0 || p.mode > 2) return DC_ERR_ARG;
  if (p.mode == 2 && p.kh != 3) return DC_ERR_ARG;
  if (d->algo < 0 || d->algo > kNumExt || d->splitk < ((d->algo > kNumAll && d->algo < kWideFirst) ? -32 : -4))
    return DC_ERR_ARG;
  const bool smallc = (p.cin % 64) != 0;
  if (d->x2 && (smallc || p.c1 % 64 != 0)) return DC_ERR_ARG;
  if ((p.ldx | p.ldx2 | p.ldy) % 8 != 0) return DC_ERR_ALIGN;
  if (p.resid && p.ldr % 8 != 0) return DC_ERR_ALIGN;
  if (p.mask && p.ldmask % 8 != 0) return DC_ERR_ALIGN;
  if (((uintptr_t)p.x | (uintptr_t)p.x2 | (uintptr_t)p.w | (uintptr_t)p.y) & 15) return DC_ERR_ALIGN;
  if (((uintptr_t)p.resid | (uintptr_t)p.mask) & 15) return DC_ERR_ALIGN;
  // 32-bit pixel arithmetic in the gather (fast_div): pixel indices, and the nearest-upsample source products
  // (output row / column index x input size, mode 1), below 2^31
  if (p.hin <= 0 || p.win <= 0 || (long)p.nb * p.hout * p.wout >= (1L << 31) ||
      (long)p.nb * p.hin * p.win >= (1L << 31))
    return DC_ERR_ARG;
  if (p.mode == 1 && ((long)p.hout * p.hin >= (1L << 31) || (long)p.wout * p.win >= (1L << 31))) return DC_ERR_ARG;
  make_fast_div((unsigned)(p.hout * p.wout), p.hw_mul, p.hw_shr);
  make_fast_div((unsigned)p.wout, p.w_mul, p.w_shr);
  make_fast_div((unsigned)p.hout, p.h_mul, p.h_shr);
  const long M = p.rows ? p.nrows : (long)p.nb * p.hout * p.wout;
  M_out = M;
  memset(&p.gn, 0, sizeof p.gn);
  if (d->gn) {
    // fused GroupNorm statistics: whole 8-channel vectors, every output row in a whole frame of each target
    const dc_gn_fuse& g = *d->gn;
    if (g.mode < 1 || g.mode > 2 || g.nt < 1 || g.nt > 2 || (g.mode == 2 && g.nt != 1)) return DC_ERR_ARG;
    if (p.rows || p.geglu || p.cout % 8) return DC_ERR_ARG;
    p.gn.mode = g.mode;
    p.gn.nt = g.nt;
    for (int k = 0; k < g.nt; ++k) {
      const dc_gn_target& t = g.t[k];
      if (!t.acc || ((uintptr_t)t.acc & 7) || t.groups <= 0 || t.groups > 64 || t.cpg <= 0 || t.hw <= 0 || t.coff < 0 ||
          t.coff % 8 || t.coff + p.cout > t.groups * t.cpg || M % t.hw)
        return DC_ERR_ARG;
      if (k > 0 && t.hw != g.t[0].hw) return DC_ERR_ARG;
      GnTargetP& q = p.gn.t[k];
      q.acc = reinterpret_cast<unsigned long long*>(t.acc);
      q.coff = t.coff;
      q.groups = t.groups;
      q.cpg = t.cpg;
      q.hw = t.hw;
      q.rstride = (M / t.hw) * t.groups * kGnPair;
      make_fast_div((unsigned)t.hw, q.hw_mul, q.hw_shr);
    }
    if (g.mode == 2) {
      // the output is the whole normalised tensor's gradient; its input x (x2: channels >= c1) is read per row
      const dc_gn_target& t = g.t[0];
      if (t.coff != 0 || t.groups * t.cpg != p.cout || !g.x || !g.stats || !g.gamma || !g.beta) return DC_ERR_ARG;
      if (g.ldx % 8 || ((uintptr_t)g.x & 15)) return DC_ERR_ALIGN;
      if (g.x2 && (g.ldx2 % 8 || g.c1 % 8 || ((uintptr_t)g.x2 & 15))) return DC_ERR_ALIGN;
      p.gn.x = (const bf16*)g.x;
      p.gn.x2 = (const bf16*)(g.x2 ? g.x2 : g.x);
      p.gn.ldx = g.ldx;
      p.gn.ldx2 = g.x2 ? g.ldx2 : g.ldx;
      p.gn.c1 = g.x2 ? g.c1 : (1 << 30);
      p.gn.stats = g.stats;
      p.gn.gamma = g.gamma;
      p.gn.beta = g.beta;
      p.gn.silu = g.silu ? 1 : 0;
    }
  }
  p.ln_csum = nullptr;
  p.ln_cbias = nullptr;
  p.ln_stats = nullptr;
  return DC_OK;
}

extern "C" int dc_conv_gemm(const dc_conv_desc* d, void* stream) {
  ConvGemmParams p;
  long M = 0;
  if (const int st = conv_params(d, p, M)) return st;
  const bool smallc = (p.cin % 64) != 0;
  hipStream_t s = (hipStream_t)stream;
  int algo = d->algo, splits = d->splitk;
  if (d->ln) {
    // LayerNorm folded in (dc_ln_fuse): a linear on an im2col tile (split-K / stream-K allowed: the epilogue
    // applies the row statistics to the summed tile)
    const dc_ln_fuse& l = *d->ln;
    if (!l.csum || !l.cbias || !l.stats || p.bias || p.gn.mode || p.rows || d->x2 || p.geglu > 1 || p.kh != 1 ||
        p.kw != 1 || p.stride != 1 || p.pad != 0 || p.mode != 0 || p.cin != p.ktot || p.hin != p.hout ||
        p.win != p.wout)
      return DC_ERR_ARG;
    p.ln_csum = l.csum;
    p.ln_cbias = l.cbias;
    p.ln_stats = l.stats;
    const bool im2col = (algo >= 1 && algo <= kNumBase) || (algo > kNumBase + kNumHalo && algo <= kNumAll);
    if (!im2col || splits == 0) {   // a halo / skinny / resident / wide choice, or none: the im2col heuristic
      int a2, s2;
      auto_algo(M, p.cout, p.ktot / 64, a2, s2);
      if (!im2col) algo = a2;
      splits = (!im2col || splits == 0) ? s2 : splits;
    }
    return conv_launch_algo_ln(algo_index(algo), p, M, splits, smallc, s);
  }
  if (algo >= kWideFirst && !algo_is_halo(algo)) {
    // wide im2col tile: the launch below (algo_index maps it into kAlgos).  No fused-GroupNorm form: a GroupNorm-fused
    // call that carries a wide choice (the table's entry is shared with the shape's unfused calls, and a shape is
    // tuned before its GroupNorm consumers register) runs the 64 x 64 double-buffered tile, the level-0 winner before
    // A folded FF2 / proj_out input-gradient (geglu_n) splits its epilogue per column tile at geglu_n, a multiple of
    // 256: a 320-wide tile can straddle it (4C = 256 / 512 for C = 64 / 128), so it takes that tile too.
    if (p.gn.mode != 0 || p.geglu_n != 0) {
      algo = 13;
      splits = 1;
    }
  } else if (algo > kNumAll + kNumSkinny && algo < kWideFirst) {
    const int ri = algo - kNumAll - kNumSkinny - 1;
    if (resident_eligible(p)) return conv_launch_resident(ri, p, splits, s);
    algo = 0;   // outside the narrow-conv contract (nearest-shape pick): im2col heuristic
    splits = 0;
  }
  if (algo > kNumAll && algo < kWideFirst) {
    const int si = algo - kNumAll - 1;
    if (skinny_eligible(p, si))
      return kSkinnyAlgos[si].kt == 9 ? conv_launch_skinny9(si, p, splits == 0 ? 1 : splits, s)
                                      : conv_launch_skinny1(si, p, splits == 0 ? 1 : splits, s);
    algo = 0;   // a skinny choice carried to a shape outside its contract (nearest-shape pick): im2col heuristic
    splits = 0;
  }
  if (algo_is_halo(algo)) {
    if (halo_eligible(p)) {
      const int hi = halo_index(algo);
      const int hs = splits == 0 ? 1 : splits;
      return p.gn.mode == 1 ? conv_launch_halo_gn(hi, p, hs, s)
           : p.gn.mode == 2 ? conv_launch_halo_gnb(hi, p, hs, s) : launch_halo_idx<0>(hi, p, hs, s);
    }
    algo = 0;   // a halo choice carried to a shape outside its contract (nearest-shape pick): im2col heuristic
    splits = 0;
  }
  if (algo == 0 || splits == 0) {
    int a2, s2;
    auto_algo(M, p.cout, p.ktot / 64, a2, s2);
    if (algo == 0) algo = a2;
    if (splits == 0) splits = (d->algo == 0) ? s2 : 1;
  }
  algo = algo_index(algo);
  return p.gn.mode == 1   ? conv_launch_algo_gn(algo, p, M, splits, smallc, s)
         : p.gn.mode == 2 ? conv_launch_algo_gnb(algo, p, M, splits, smallc, s)
                          : launch_algo_idx<0>(algo, p, M, splits, smallc, s);
}

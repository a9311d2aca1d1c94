// Folded 2-key cross-attention (attn2 of the UNet's BasicTransformerBlocks with the constant empty-prompt
// context, marigold_dc.py:463, 663-674) fused with its LayerNorm (norm2) and residual, on MFMA (gfx950).
//
//   out = x + c0 + sum_h sigmoid(LN2(x) . U_h) D_h          (U, D: [H][C] fp32, c0: [C])
//
// is a rank-H bottleneck [rows x C] -> [rows x H] -> [rows x C].  Per row it needs every element of U and D
// (12.8 KB at C 320 x 5 heads, 204 KB at 1280 x 20), so a one-row-per-wave form re-reads the whole tables for
// every row.  Here a block takes 16 rows and both contractions run as v_mfma_f32_16x16x32_bf16 tiles, so every
// table element read serves 16 rows:
//   logits [16 x 32] = LN(x) [16 x C] . U^T        (K = C split over the block's waves, partials summed in LDS)
//   out    [16 x C]  = sigmoid(logits) . D          (K = 32 padded heads, N = C split over the waves)
// LN(x) is exactly bf16 (the reference rounds the LayerNorm output), so the first A operand is exact; the
// fp32 tables and sigmoids enter as bf16 hi + lo pairs (hi = bf16(v), lo = bf16(v - hi): 16 mantissa bits), the
// logits with 2 MFMAs (hi, lo) and the output with 3 (hi.hi + hi.lo + lo.hi) -- ~2^-16 relative, far inside
// the reference's own bf16 rounding of q / k / v / P.  The backward is the same two contractions transposed
// (G = dy . D^T, dn = (G * p(1 - p)) . U) followed by the LayerNorm backward.
//
// Tables (dc_crossattn_prepare, once at load time; 8 x 32 x C bf16): UH, UL, DH, DL [32][C] (B operands of the
// K = C contractions: 8 contiguous channels per lane) and DTH, DTL, UTH, UTL [C][32] (B operands of the K = heads
// contractions: 8 contiguous heads per lane); padded heads are zero.
// Latency: a block of 16 rows runs 8 waves (C <= 1024) or 16 (C = 1280), each owning a few channel chunks and
// output column tiles, with every global load of the wave issued before its first MFMA, so the block pays about
// one memory round trip per phase (a 4-wave form with ~20 dependent table loads per wave took 20-35 us at
// 432 x 1280 whatever the row count).
#include "common.h"
#include "../../include/dcamd.h"

namespace {

constexpr int kHP = 32;        // padded heads (H <= 20 in the SD2 UNet)
constexpr int kRows = 16;      // rows per block (one MFMA M tile)
// per-wave maxima by block width (register budget: 16-wave blocks are capped at 128 VGPRs):
//   NW  8: <= 2 channel chunks, <= 3 column tiles -> C <= 384  (UNet level 0: 320)
//   NW 16: <= 3 channel chunks, <= 5 column tiles -> C <= 1280 (levels 1-3: 640, 1280)
template <int NW> struct Fit;
template <> struct Fit<8> { static constexpr int MK = 2, MCT = 3, MAXC = 384; };
template <> struct Fit<16> { static constexpr int MK = 3, MCT = 5, MAXC = 1280; };
// per-channel vectors (gamma, beta, c0) staged in LDS: elements per thread of the block-cooperative load
template <int NW> constexpr int kStage = (Fit<NW>::MAXC + 64 * NW - 1) / (64 * NW);
constexpr int kMaxC = 1280;

__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bf16 h = (bf16)v[j];
    hi[j] = h;
    lo[j] = (bf16)(v[j] - (float)h);
  }
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// row sum over the 4 lane groups of a wave (lanes r, r + 16, r + 32, r + 48 hold row r)
__device__ __forceinline__ float rowsum4(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
// sum over the 16 lanes of a lane group (the columns of a C-layout tile)
__device__ __forceinline__ float colsum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct Tabs {
  const bf16 *uh, *ul, *dh, *dl, *dth, *dtl, *uth, *utl;
  __device__ Tabs(const bf16* t, int c) {
    const long s = (long)kHP * c;
    uh = t; ul = t + s; dh = t + 2 * s; dl = t + 3 * s; dth = t + 4 * s; dtl = t + 5 * s; uth = t + 6 * s; utl = t + 7 * s;
  }
};

__global__ void cross_prepare_kernel(const float* U, const float* D, int heads, int c, bf16* tabs) {
  const long s = (long)kHP * c;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < s; i += (long)gridDim.x * blockDim.x) {
    const int h = (int)(i / c), ch = (int)(i - (long)h * c);
    const float u = h < heads ? U[(long)h * c + ch] : 0.0f;
    const float d = h < heads ? D[(long)h * c + ch] : 0.0f;
    const bf16 uh = (bf16)u, dh = (bf16)d;
    const bf16 ul = (bf16)(u - (float)uh), dl = (bf16)(d - (float)dh);
    tabs[i] = uh;                               // [h][c]
    tabs[s + i] = ul;
    tabs[2 * s + i] = dh;
    tabs[3 * s + i] = dl;
    const long t = (long)ch * kHP + h;          // [c][h]
    tabs[4 * s + t] = dh;
    tabs[5 * s + t] = dl;
    tabs[6 * s + t] = uh;
    tabs[7 * s + t] = ul;
  }
}

// K = C contraction of the wave's channel chunks [kb, ke): acc[ht] += A (16 rows x 32 ch) . B^T (32 ch x 16 heads),
// B = (hi, lo) tables [32][C]; the B fragments are loaded (load_k) before the A operands are ready
template <int MK>
__device__ __forceinline__ void load_k(int kb, int ke, const bf16* bh, const bf16* bl, int c, int r, int g,
                                       bf16x8 (&b)[MK][2][2]) {
#pragma unroll
  for (int i = 0; i < MK; ++i)
    if (kb + i < ke)
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        const long off = (long)(ht * 16 + r) * c + (kb + i) * 32 + g * 8;
        b[i][ht][0] = ld8(bh + off);
        b[i][ht][1] = ld8(bl + off);
      }
}
template <int MK>
__device__ __forceinline__ void contract_k(const bf16x8 (&a)[MK], int kb, int ke, const bf16x8 (&b)[MK][2][2],
                                           f32x4 (&acc)[2]) {
#pragma unroll
  for (int i = 0; i < MK; ++i)
    if (kb + i < ke)
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        acc[ht] = mfma(a[i], b[i][ht][0], acc[ht]);
        acc[ht] = mfma(a[i], b[i][ht][1], acc[ht]);
      }
}

// B fragments (hi, lo) of the K = heads contraction for the wave's column tiles [cb, ce), table [C][32]
template <int MCT>
__device__ __forceinline__ void load_ct(const bf16* th, const bf16* tl, int cb, int ce, int r, int g,
                                        bf16x8 (&b)[MCT][2]) {
#pragma unroll
  for (int t = 0; t < MCT; ++t)
    if (cb + t < ce) {
      const long off = (long)((cb + t) * 16 + r) * kHP + g * 8;
      b[t][0] = ld8(th + off);
      b[t][1] = ld8(tl + off);
    }
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void cross_mfma_fwd_kernel(const bf16* x, int ldx, long rows, int c, int heads,
                                                                 float eps, const float* gamma, const float* beta,
                                                                 const bf16* tabs, const float* c0, bf16* y, int ldy,
                                                                 float* stats, float* probs, float* ystats, float yeps) {
  constexpr int MK = Fit<NW>::MK, MCT = Fit<NW>::MCT;
  __shared__ float s_red[NW][kRows];
  __shared__ float s_part[NW][kRows][kHP + 1];
  __shared__ float s_sig[kRows][kHP + 4];
  __shared__ float s_tile[NW][kRows][17];
  // gamma, beta, c0 staged once per block: read from global memory inside the phases below they were dependent
  // round trips, one per channel chunk (gamma, beta) and one per column tile (c0)
  __shared__ float s_aff[3][Fit<NW>::MAXC];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const long row0 = (long)blockIdx.x * kRows;
  const long row = row0 + r;
  const bool ok = row < rows;
  const int nk = c >> 5, kb = w * nk / NW, ke = (w + 1) * nk / NW;
  const int nct = c >> 4, cb = w * nct / NW, ce = (w + 1) * nct / NW;
  const int rr = lane >> 2, cc = (lane & 3) * 4;  // write-back mapping: row rr, columns cc .. cc + 3 of a tile
  const long orow = row0 + rr;
  const Tabs T(tabs, c);

  // phase 1: x chunks and the logits tables in flight together; LayerNorm statistics (two-pass, fp32, the
  // waves' partials folded in wave order)
  // every load unconditional (a row past the end reads the last row; nothing of it is stored): a load guarded by a
  // lane condition sits in a divergent branch, and the compiler waits for it before leaving the branch
  const long rowc = ok ? row : rows - 1;
  // (chunks past the wave's last -- all of them for a wave without chunks, C < 32 NW -- re-read the row's last chunk and
  // are skipped at every use)
  bf16x8 xv[MK];
#pragma unroll
  for (int i = 0; i < MK; ++i) xv[i] = ld8(x + rowc * ldx + min(kb + i, nk - 1) * 32 + g * 8);
  bf16x8 bk[MK][2][2];
  load_k<MK>(kb, ke, T.uh, T.ul, c, r, g, bk);
  float aff[3][kStage<NW>];
#pragma unroll
  for (int k = 0; k < kStage<NW>; ++k) {
    const int i = min((int)threadIdx.x + 64 * NW * k, c - 1);
    aff[0][k] = gamma[i];
    aff[1][k] = beta[i];
    aff[2][k] = c0[i];
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < MK; ++i)
    if (kb + i < ke)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += (float)xv[i][j];
  s = rowsum4(s);
  if (g == 0) s_red[w][r] = s;
#pragma unroll
  for (int k = 0; k < kStage<NW>; ++k) {
    const int i = threadIdx.x + 64 * NW * k;
    if (i < c) {
      s_aff[0][i] = aff[0][k];
      s_aff[1][i] = aff[1][k];
      s_aff[2][i] = aff[2][k];
    }
  }
  __syncthreads();
  float tot = 0.0f;
#pragma unroll
  for (int v = 0; v < NW; ++v) tot += s_red[v][r];
  const float mu = tot / c;
  __syncthreads();
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < MK; ++i)
    if (kb + i < ke)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (float)xv[i][j] - mu;
        q += d * d;
      }
  q = rowsum4(q);
  if (g == 0) s_red[w][r] = q;
  __syncthreads();
  tot = 0.0f;
#pragma unroll
  for (int v = 0; v < NW; ++v) tot += s_red[v][r];
  const float rs = rsqrtf(tot / c + eps);
  // phase 2: LN2(x) rounded to bf16 (exact MFMA operand, in place) and the logits partials
#pragma unroll
  for (int i = 0; i < MK; ++i) {
    if (kb + i < ke) {
      const int ch = (kb + i) * 32 + g * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[i][j] = (bf16)(((float)xv[i][j] - mu) * rs * s_aff[0][ch + j] + s_aff[1][ch + j]);
    }
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  contract_k<MK>(xv, kb, ke, bk, acc);
  // the output tables and the residual rows load while the logits are folded
  bf16x8 bt[MCT][2];
  load_ct<MCT>(T.dth, T.dtl, cb, ce, r, g, bt);
  bf16x4 xres[MCT];
#pragma unroll
  for (int t = 0; t < MCT; ++t)
    if (cb + t < ce && orow < rows) xres[t] = *reinterpret_cast<const bf16x4*>(x + orow * ldx + (cb + t) * 16 + cc);
#pragma unroll
  for (int ht = 0; ht < 2; ++ht)
#pragma unroll
    for (int e = 0; e < 4; ++e) s_part[w][g * 4 + e][ht * 16 + r] = acc[ht][e];
  if (w == 0 && g == 0 && ok) {
    stats[row * 2] = mu;
    stats[row * 2 + 1] = rs;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kRows * kHP; i += 64 * NW) {
    const int ro = i / kHP, hh = i - ro * kHP;
    float lg = 0.0f;
#pragma unroll
    for (int v = 0; v < NW; ++v) lg += s_part[v][ro][hh];
    const float p = hh < heads ? 1.0f / (1.0f + __expf(-lg)) : 0.0f;
    s_sig[ro][hh] = p;
    if (hh < heads && row0 + ro < rows) probs[(row0 + ro) * heads + hh] = p;
  }
  __syncthreads();
  // phase 3: out tiles, A = sigmoid (rows x 32 heads) as hi / lo, B = D^T (32 heads x 16 columns)
  bf16x8 sh, sl;
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = s_sig[r][g * 8 + j];
    split8(v, sh, sl);
  }
  float yv[MCT][4];   // the stored output values of the lane's row segments (norm3's statistics below)
#pragma unroll
  for (int t = 0; t < MCT; ++t) {
    const int ct = cb + t;
#pragma unroll
    for (int j = 0; j < 4; ++j) yv[t][j] = 0.0f;
    if (ct < ce) {
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
      o = mfma(sh, bt[t][0], o);
      o = mfma(sh, bt[t][1], o);
      o = mfma(sl, bt[t][0], o);
      const float cv = s_aff[2][ct * 16 + r];
#pragma unroll
      for (int e = 0; e < 4; ++e) s_tile[w][g * 4 + e][r] = (float)(bf16)(o[e] + cv);
      __builtin_amdgcn_wave_barrier();
      if (orow < rows) {
        bf16x4 ov;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ov[j] = (bf16)(s_tile[w][rr][cc + j] + (float)xres[t][j]);
          yv[t][j] = (float)ov[j];
        }
        *reinterpret_cast<bf16x4*>(y + orow * ldy + ct * 16 + cc) = ov;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (ystats) {
    // (mean, rstd) of each output row (the next LayerNorm's statistics, dc_ln_fuse): two passes over the stored
    // values, the 4 lanes of a row then the waves in order
    float sm = 0.0f;
#pragma unroll
    for (int t = 0; t < MCT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) sm += yv[t][j];
    sm += __shfl_xor(sm, 1, 64);
    sm += __shfl_xor(sm, 2, 64);
    __syncthreads();
    if ((lane & 3) == 0) s_red[w][rr] = sm;
    __syncthreads();
    float tot = 0.0f;
#pragma unroll
    for (int v = 0; v < NW; ++v) tot += s_red[v][rr];
    const float ym = tot / c;
    float q = 0.0f;
#pragma unroll
    for (int t = 0; t < MCT; ++t)
      if (cb + t < ce)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = yv[t][j] - ym;
          q += d * d;
        }
    q += __shfl_xor(q, 1, 64);
    q += __shfl_xor(q, 2, 64);
    __syncthreads();
    if ((lane & 3) == 0) s_red[w][rr] = q;
    __syncthreads();
    tot = 0.0f;
#pragma unroll
    for (int v = 0; v < NW; ++v) tot += s_red[v][rr];
    if (w == 0 && (lane & 3) == 0 && orow < rows) {
      ystats[orow * 2] = ym;
      ystats[orow * 2 + 1] = rsqrtf(tot / c + yeps);
    }
  }
}

// The LayerNorm (norm3) backward that produces this kernel's dy, fused in front of it (LN3 = true): dy = LN3bwd(dl) +
// add for the block's 16 rows into an LDS tile, one wave per row, with the arithmetic (and summation order) of
// norms.hip ln_bwd_kernel with gamma folded into dl (dc_ln_fuse) -- the same bits as the two-launch form.
struct Ln3Bwd {
  const bf16* dl;
  int lddl;
  const bf16* x3;   // norm3's input (r2)
  int ldx3;
  const float* stats3;
  const bf16* add;
  int ldadd;
};
constexpr int kDyLd = kMaxC + 8;   // LDS row stride of the dy tile (bf16; 16-B pad against bank conflicts)

template <int MAXV>
__device__ __forceinline__ void ln3_bwd_row(const Ln3Bwd& L, long row, int c, int lane, bf16* out) {
  const int nv = c >> 3;
  const float mu = L.stats3[row * 2], rs = L.stats3[row * 2 + 1];
  // the row's loads all issued up front, the residual addend included (clamped segments, skipped below): read after
  // the row sums, the addend was a second dependent round trip
  bf16x8 xr[MAXV], dr[MAXV], ar[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vc = min(lane + 64 * k, nv - 1);
    xr[k] = ld8(L.x3 + row * L.ldx3 + vc * 8);
    dr[k] = ld8(L.dl + row * L.lddl + vc * 8);
    ar[k] = ld8(L.add + row * L.ldadd + vc * 8);
  }
  float xh[MAXV][8], gg[MAXV][8];
  float sa = 0.0f, sb = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[k][i] = ((float)xr[k][i] - mu) * rs;
        gg[k][i] = (float)dr[k][i];
        sa += gg[k][i];
        sb += gg[k][i] * xh[k][i];
      }
    }
  }
  const float ma = wave_sum(sa) / c, mb = wave_sum(sb) / c;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (float)(bf16)(rs * (gg[k][i] - ma - xh[k][i] * mb)) + (float)ar[k][i];
      store8(out + vi * 8, o);
    }
  }
}

template <int NW, bool LN3>
__global__ __launch_bounds__(64 * NW) void cross_mfma_bwd_kernel(const bf16* x, int ldx, long rows, int c, int heads,
                                                                 const float* gamma, const bf16* tabs,
                                                                 const float* stats, const float* probs, const bf16* dy,
                                                                 int lddy, bf16* dx, int lddx, Ln3Bwd ln3) {
  constexpr int MK = Fit<NW>::MK, MCT = Fit<NW>::MCT;
  __shared__ float s_part[NW][kRows][kHP + 1];
  __shared__ float s_sig[kRows][kHP + 4];
  __shared__ float s_red[NW][kRows][2];
  __shared__ float s_tile[NW][kRows][17];
  __shared__ __attribute__((aligned(16))) bf16 s_dy[LN3 ? kRows : 1][LN3 ? kDyLd : 8];
  // gamma and the block's probabilities staged once (as in the forward: per-tile / post-barrier global reads were
  // dependent round trips)
  __shared__ float s_gam[Fit<NW>::MAXC];
  __shared__ float s_prob[kRows][kHP];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const long row0 = (long)blockIdx.x * kRows;
  const long row = row0 + r;
  const bool ok = row < rows;
  const int nk = c >> 5, kb = w * nk / NW, ke = (w + 1) * nk / NW;
  const int nct = c >> 4, cb = w * nct / NW, ce = (w + 1) * nct / NW;
  const int rr = lane >> 2, cc = (lane & 3) * 4;
  const long orow = row0 + rr;
  const Tabs T(tabs, c);
  float gst[kStage<NW>];
#pragma unroll
  for (int k = 0; k < kStage<NW>; ++k) gst[k] = gamma[min((int)threadIdx.x + 64 * NW * k, c - 1)];
  static_assert(64 * NW >= kRows * kHP, "one staged probability per thread");
  const int pro = threadIdx.x / kHP, phh = threadIdx.x - pro * kHP;
  const float pst = probs[min((row0 + min(pro, kRows - 1)) * heads + min(phh, heads - 1), rows * heads - 1)];
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < kStage<NW>; ++k) {
      const int i = threadIdx.x + 64 * NW * k;
      if (i < c) s_gam[i] = gst[k];
    }
    if (pro < kRows) s_prob[pro][phh] = pst;
  };
  if constexpr (LN3) {
    // phase 0: dy of the block's rows (norm3 backward + residual) into the LDS tile
    for (int q = w; q < kRows; q += NW) {
      if (row0 + q < rows) {
        if ((c >> 3) <= 64) ln3_bwd_row<1>(ln3, row0 + q, c, lane, &s_dy[q][0]);
        else ln3_bwd_row<3>(ln3, row0 + q, c, lane, &s_dy[q][0]);
      }
    }
    stage();
    __syncthreads();
  }
  // dy row r / rr of the block: the LDS tile (LN3) or global memory
  auto dy_at = [&](int rl, long rg, int col) -> const bf16* {
    if constexpr (LN3) return &s_dy[rl][col];
    else return dy + rg * lddy + col;
  };
  // phase 1: G = dy . D^T over the wave's channel chunks (dy is exactly bf16)
  bf16x8 av[MK];   // unconditional loads, chunks past the wave's last skipped at their use (see the forward)
#pragma unroll
  for (int i = 0; i < MK; ++i) av[i] = ld8(dy_at(r, ok ? row : rows - 1, min(kb + i, nk - 1) * 32 + g * 8));
  bf16x8 bk[MK][2][2];
  load_k<MK>(kb, ke, T.dh, T.dl, c, r, g, bk);
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  contract_k<MK>(av, kb, ke, bk, acc);
  // the dn tables and the row-major x / dy segments of the write-back load while G is folded
  bf16x8 bt[MCT][2];
  load_ct<MCT>(T.uth, T.utl, cb, ce, r, g, bt);
  bf16x4 xw[MCT], dyw[MCT];
#pragma unroll
  for (int t = 0; t < MCT; ++t)
    if (cb + t < ce && orow < rows) {
      xw[t] = *reinterpret_cast<const bf16x4*>(x + orow * ldx + (cb + t) * 16 + cc);
      dyw[t] = *reinterpret_cast<const bf16x4*>(dy_at(rr, orow, (cb + t) * 16 + cc));
    }
  const float mu = orow < rows ? stats[orow * 2] : 0.0f;
  const float rs = orow < rows ? stats[orow * 2 + 1] : 0.0f;
#pragma unroll
  for (int ht = 0; ht < 2; ++ht)
#pragma unroll
    for (int e = 0; e < 4; ++e) s_part[w][g * 4 + e][ht * 16 + r] = acc[ht][e];
  if constexpr (!LN3) stage();
  __syncthreads();
  for (int i = threadIdx.x; i < kRows * kHP; i += 64 * NW) {
    const int ro = i / kHP, hh = i - ro * kHP;
    float gs = 0.0f;
#pragma unroll
    for (int v = 0; v < NW; ++v) gs += s_part[v][ro][hh];
    float dsg = 0.0f;
    if (hh < heads && row0 + ro < rows) {
      const float p = s_prob[ro][hh];
      dsg = gs * p * (1.0f - p);
    }
    s_sig[ro][hh] = dsg;
  }
  __syncthreads();
  bf16x8 sh, sl;
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = s_sig[r][g * 8 + j];
    split8(v, sh, sl);
  }
  // phase 2: dn = dsg . U through the per-wave LDS tile into the row-major mapping, rounded to bf16, times gamma;
  // LayerNorm-backward row sums over the wave's columns
  float dn[MCT][4];
  float sa = 0.0f, sb = 0.0f;
#pragma unroll
  for (int t = 0; t < MCT; ++t) {
    const int ct = cb + t;
    if (ct < ce) {
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
      o = mfma(sh, bt[t][0], o);
      o = mfma(sh, bt[t][1], o);
      o = mfma(sl, bt[t][0], o);
#pragma unroll
      for (int e = 0; e < 4; ++e) s_tile[w][g * 4 + e][r] = o[e];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = ct * 16 + cc + j;
        const float xh = ((float)xw[t][j] - mu) * rs;
        dn[t][j] = (float)(bf16)s_tile[w][rr][cc + j] * s_gam[col];
        if (orow < rows) {
          sa += dn[t][j];
          sb += dn[t][j] * xh;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  // row sums: the 4 lanes sharing a row (lanes 4 rr .. 4 rr + 3), then the waves in order
  sa += __shfl_xor(sa, 1, 64);
  sa += __shfl_xor(sa, 2, 64);
  sb += __shfl_xor(sb, 1, 64);
  sb += __shfl_xor(sb, 2, 64);
  if ((lane & 3) == 0) {
    s_red[w][rr][0] = sa;
    s_red[w][rr][1] = sb;
  }
  __syncthreads();
  float ta = 0.0f, tb = 0.0f;
#pragma unroll
  for (int v = 0; v < NW; ++v) {
    ta += s_red[v][rr][0];
    tb += s_red[v][rr][1];
  }
  const float ma = ta / c, mb = tb / c;
  if (orow < rows) {
#pragma unroll
    for (int t = 0; t < MCT; ++t) {
      const int ct = cb + t;
      if (ct < ce) {
        bf16x4 ov;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = ((float)xw[t][j] - mu) * rs;
          ov[j] = (bf16)((float)(bf16)(rs * (dn[t][j] - ma - xh * mb)) + (float)dyw[t][j]);
        }
        *reinterpret_cast<bf16x4*>(dx + orow * lddx + ct * 16 + cc) = ov;
      }
    }
  }
}

// waves per block (Fit): 8 up to C = 384, 16 up to C = 1280
inline int cross_waves(int c) { return c <= 384 ? 8 : 16; }

}  // namespace

extern "C" long long dc_crossattn_tables_bytes(int heads, int c) {
  if (heads <= 0 || heads > kHP || c <= 0) return 0;
  return 8LL * kHP * c * 2;
}

extern "C" int dc_crossattn_prepare(const float* U, const float* D, int heads, int c, void* tabs, void* stream) {
  if (!U || !D || !tabs || heads <= 0 || heads > kHP || c % 32 || c > kMaxC) return DC_ERR_ARG;
  const long s = (long)kHP * c;
  hipLaunchKernelGGL(cross_prepare_kernel, dim3((unsigned)((s + 255) / 256)), dim3(256), 0, (hipStream_t)stream, U, D,
                     heads, c, (bf16*)tabs);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_crossattn_fwd(const void* x, int ldx, long long rows, int c, int heads, float eps,
                                const float* gamma, const float* beta, const void* tabs, const float* c0, void* y,
                                int ldy, float* stats, float* probs, float* ystats, float yeps, void* stream) {
  if (!x || !y || !gamma || !beta || !tabs || !c0 || !stats || !probs || rows <= 0 || heads <= 0 || heads > kHP ||
      c % 32 || c > kMaxC)
    return DC_ERR_ARG;
  if (ldx % 8 || ldy % 8 || ((uintptr_t)x & 15) || ((uintptr_t)y & 7)) return DC_ERR_ALIGN;
  const dim3 grid((unsigned)((rows + kRows - 1) / kRows));
  if (cross_waves(c) == 8)
    hipLaunchKernelGGL(cross_mfma_fwd_kernel<8>, grid, dim3(512), 0, (hipStream_t)stream, (const bf16*)x, ldx,
                       (long)rows, c, heads, eps, gamma, beta, (const bf16*)tabs, c0, (bf16*)y, ldy, stats, probs,
                       ystats, yeps);
  else
    hipLaunchKernelGGL(cross_mfma_fwd_kernel<16>, grid, dim3(1024), 0, (hipStream_t)stream, (const bf16*)x, ldx,
                       (long)rows, c, heads, eps, gamma, beta, (const bf16*)tabs, c0, (bf16*)y, ldy, stats, probs,
                       ystats, yeps);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

namespace {
template <bool LN3>
int cross_bwd_launch(const void* x, int ldx, long long rows, int c, int heads, const float* gamma, const void* tabs,
                     const float* stats, const float* probs, const void* dy, int lddy, void* dx, int lddx,
                     const Ln3Bwd& ln3, void* stream) {
  const dim3 grid((unsigned)((rows + kRows - 1) / kRows));
  if (cross_waves(c) == 8)
    hipLaunchKernelGGL((cross_mfma_bwd_kernel<8, LN3>), grid, dim3(512), 0, (hipStream_t)stream, (const bf16*)x, ldx,
                       (long)rows, c, heads, gamma, (const bf16*)tabs, stats, probs, (const bf16*)dy, lddy, (bf16*)dx,
                       lddx, ln3);
  else
    hipLaunchKernelGGL((cross_mfma_bwd_kernel<16, LN3>), grid, dim3(1024), 0, (hipStream_t)stream, (const bf16*)x,
                       ldx, (long)rows, c, heads, gamma, (const bf16*)tabs, stats, probs, (const bf16*)dy, lddy,
                       (bf16*)dx, lddx, ln3);
  DC_CHECK_LAUNCH();
  return DC_OK;
}
}  // namespace

extern "C" int dc_crossattn_bwd(const void* x, int ldx, long long rows, int c, int heads, const float* gamma,
                                const void* tabs, const float* stats, const float* probs, const void* dy, int lddy,
                                void* dx, int lddx, void* stream) {
  if (!x || !dy || !dx || !gamma || !tabs || !stats || !probs || rows <= 0 || heads <= 0 || heads > kHP || c % 32 ||
      c > kMaxC)
    return DC_ERR_ARG;
  if (ldx % 8 || lddy % 8 || lddx % 8 || ((uintptr_t)dy & 15) || ((uintptr_t)x & 7) || ((uintptr_t)dx & 7))
    return DC_ERR_ALIGN;
  return cross_bwd_launch<false>(x, ldx, rows, c, heads, gamma, tabs, stats, probs, dy, lddy, dx, lddx, Ln3Bwd{},
                                 stream);
}

extern "C" int dc_crossattn_bwd_ln(const void* x, int ldx, long long rows, int c, int heads, const float* gamma,
                                   const void* tabs, const float* stats, const float* probs, const void* dl, int lddl,
                                   const void* x3, int ldx3, const float* stats3, const void* add, int ldadd, void* dx,
                                   int lddx, void* stream) {
  if (!x || !dl || !x3 || !stats3 || !add || !dx || !gamma || !tabs || !stats || !probs || rows <= 0 || heads <= 0 ||
      heads > kHP || c % 32 || c > kMaxC)
    return DC_ERR_ARG;
  if (ldx % 8 || lddl % 8 || ldx3 % 8 || ldadd % 8 || lddx % 8 || ((uintptr_t)dl & 15) || ((uintptr_t)x3 & 15) ||
      ((uintptr_t)add & 15) || ((uintptr_t)x & 7) || ((uintptr_t)dx & 7))
    return DC_ERR_ALIGN;
  const Ln3Bwd ln3{(const bf16*)dl, lddl, (const bf16*)x3, ldx3, stats3, (const bf16*)add, ldadd};
  return cross_bwd_launch<true>(x, ldx, rows, c, heads, gamma, tabs, stats, probs, nullptr, 0, dx, lddx, ln3, stream);
}

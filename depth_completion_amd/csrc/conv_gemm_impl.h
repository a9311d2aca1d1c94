#pragma once
// Implicit-GEMM convolution / linear layer on gfx950 MFMA (v_mfma_f32_16x16x32_bf16): kernels and launchers,
// included by conv_gemm.hip (plain epilogues, the C ABI) and conv_gemm_gn.hip (fused GroupNorm statistics).
//
// One kernel family serves every matmul-shaped op of the hot path:
//   * 3x3 / 1x1 convs of the UNet resnets and TAESD (fwd), stride 2 (Downsample2D),
//     nearest-upsample folded into the A-operand addressing (Upsample2D, TAESD Upsample),
//   * their input gradients (dgrad = conv with pre-flipped/transposed weights; mode 2 is
//     the transposed stride-2 gather for the Downsample2D VJP),
//   * every nn.Linear (1x1 conv over token rows).
// GEMM view: M = output pixels (NHWC rows), N = output channels, K = taps x Cin (K contiguous in
// both operands).  Tiles BM x BN x 64 on 4 waves (2x2).  Operands are gathered straight into an
// S-deep LDS ring with global_load_lds_dwordx4 (per-lane source address = the im2col gather; padding
// and tails read a zero line), XOR-swizzled through the source permutation so the ds_read_b128
// fragment reads are conflict-free; S-2 k-chunks stay in flight across the (raw) barrier under a
// counted vmcnt.  The epilogue stages the fp32 tile through LDS and applies bias / per-step row bias
// (time embedding) / residual / ReLU / ReLU-backward mask with 16-B coalesced accesses.  Work
// decomposition: plain tiles, split-K, or stream-K (equal contiguous ranges of the tile x k-chunk
// iteration space per block); a tile computed in pieces is summed in piece order by its
// last-arriving block (deterministic, no second kernel).
#include <string.h>
#include <type_traits>
#include <utility>

#include "common.h"
#include "gn_acc.h"
#include "../../include/dcamd.h"

// fused GroupNorm statistics (dc_gn_fuse): one normalised tensor this output feeds
struct GnTargetP {
  unsigned long long* acc;
  long rstride;      // words per accumulator replica (gn_acc.h kGnReplicas)
  int coff, groups, cpg, hw;
  unsigned hw_mul;   // fast_div by hw (frame of an output row)
  int hw_shr;
};
struct GnFuseP {
  int mode, nt;      // mode 0: none
  GnTargetP t[2];
  const bf16* x;     // backward: the GroupNorm input (channels >= c1 from x2)
  const bf16* x2;
  int ldx, ldx2, c1;
  const float* stats;
  const float* gamma;
  const float* beta;
  int silu;
};

struct ConvGemmParams {
  const bf16* x;
  const bf16* x2;       // channels >= c1 come from x2 (two-source concat, UNet skip connections)
  int ldx, ldx2, c1;
  int nb, hin, win, cin;
  int hout, wout;
  int kh, kw, stride, pad;
  int mode;             // 0: direct conv; 1: nearest-upsample (hin->hout) then conv s1; 2: transposed s2 gather
  const bf16* w;        // [cout][ktot]
  int ktot, cout;
  const float* bias;    // [cout]
  const bf16* rowbias;  // [*][rowbias_ld], row selected by *rowbias_idx (per-step time embedding)
  const int* rowbias_idx;
  int rowbias_ld;
  const bf16* resid;
  int ldr;
  const bf16* mask;     // ReLU backward: out *= (mask > 0)
  int ldmask;
  int act;              // 0 none, 1 relu
  bf16* y;
  int ldy;
  float* ws;            // split-K partial slabs [splits][tiles][BM*BN]; tile counters in the last 64 KB
  long ws_bytes;
  int splits, kps;       // split-K: splits, k-chunks per split; stream-K: tile count, nk
  int* counters;        // [tiles] arrival counts, zero between launches (the workspace starts zeroed)
  int sk_blocks;        // > 0: stream-K over this many blocks (split-K / plain tiles: 0)
  int geglu;            // GEGLU epilogue (include/dcamd.h): 0 none, 1 fwd (interleaved h/gate), 2 bwd
  int geglu_n;          // geglu 2: columns >= geglu_n (> 0) are stored plainly into y2 (dc_fold_linear_pair's dgrad)
  bf16* y2;
  int ldy2;
  const bf16* aux;
  int ldaux;
  const int* rows;      // optional: GEMM row m computes output pixel rows[m] (sorted), nrows of them
  long nrows;
  int diag;             // kernel diagnostics (env DC_HALO_DIAG, experiments only): halo 1 no LDS-DMA, 2 no MFMA
                        // / fragment reads, 4 no barrier; 8 no GroupNorm-statistics accumulator adds; 256 epilogue
                        // operands loaded in the epilogue (the round-3 placement, A/B)
  int nmajor;           // tile order within an XCD's range: 0 M-major (row tiles share A), 1 N-major (column
                        // tiles share W; opt-in, DC_GEMM_ORDER=2)
  // multiply-shift division by hout * wout, wout and hout (fast_div): the pixel -> (frame, y, x) split of
  // every gathered A row in the prologue is 2 VALU per division instead of a 64-bit division sequence
  unsigned hw_mul, w_mul, h_mul;
  int hw_shr, w_shr, h_shr;
  GnFuseP gn;
  // LayerNorm of the A rows folded into a linear (dc_ln_fuse; the GNM == 3 instantiations): the epilogue applies
  // y = rstd (acc - mean csum[n]) + cbias[n] with the rows' (mean, rstd) from ln_stats
  const float* ln_csum;
  const float* ln_cbias;
  const float* ln_stats;
};

// x / d for x < 2^31 by a host-computed (mul, shr) pair (make_fast_div); mul == 0 encodes d == 1
__device__ __forceinline__ unsigned fast_div(unsigned x, unsigned mul, int shr) {
  return mul ? (__umulhi(x, mul) >> shr) : x;
}
// (mul, shr) with x / d == umulhi(x, mul) >> shr for every x < 2^31, 1 <= d < 2^31 (round-up reciprocal
// with p = 31 + ceil(log2 d): the error term stays below 2^-31 of the quotient step)
static void make_fast_div(unsigned d, unsigned& mul, int& shr) {
  if (d <= 1) {
    mul = 0;
    shr = 0;
    return;
  }
  int l = 0;
  while ((1u << l) < d) ++l;
  const int pw = 31 + l;
  mul = (unsigned)(((1ull << pw) + d - 1) / d);
  shr = pw - 32;
}

// tile index -> (row tile, column tile) in the launch's rasterisation order
__device__ __forceinline__ void tile_coords(const ConvGemmParams& p, int tile, int tiles_m, int tiles_n, int& tm,
                                            int& tn) {
  if (p.nmajor) {
    tn = tile / tiles_m;
    tm = tile - tn * tiles_m;
  } else {
    tm = tile / tiles_n;
    tn = tile - tm * tiles_n;
  }
}

// GEMM rows of the launch, and the output pixel of GEMM row m (m < conv_rows(p))
__device__ __forceinline__ long conv_rows(const ConvGemmParams& p) {
  return p.rows ? p.nrows : (long)p.nb * p.hout * p.wout;
}
__device__ __forceinline__ long conv_pix(const ConvGemmParams& p, long m) { return p.rows ? (long)p.rows[m] : m; }

static __device__ __attribute__((aligned(16))) uint4 g_zero_line[4];  // source of every padded / out-of-range piece

namespace {

// 16-B buffer stores / loads with the sc1 cache policy (device-coherent hand-off between workgroups);
// the buffer builtins keep the compiler's vmcnt tracking (an inline-asm load would not)
constexpr int kSc1 = 16;  // CPol::SC1 on gfx94x/gfx950
// raw buffer resource over [base, base + 2 GiB); the base goes through readfirstlane so the compiler
// keeps the descriptor in SGPRs (a VGPR descriptor turns every buffer access into a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  const unsigned long long a = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(float* base) { return buf_rsrc(base); }
// 16-B LDS-DMA piece: buffer_load_dwordx4 ... lds.  (The builtin only exists for the device pass; in the
// host pass of a __global__ template it silently drops the kernel's launch stub, hence the guard.)
__device__ __forceinline__ void buf_load_lds16(__amdgpu_buffer_rsrc_t r, DC_LDS char* dst, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
#endif
}
__device__ __forceinline__ void store_sc1_x4(__amdgpu_buffer_rsrc_t r, long off_f, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(off_f * 4), 0, kSc1);
}
__device__ __forceinline__ f32x4 load_sc1_x4(__amdgpu_buffer_rsrc_t r, long off_f) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off_f * 4), 0, kSc1);
}

__device__ __forceinline__ void epilogue_store(const ConvGemmParams& p, long m, int c, float* v, bool add_bias) {
  const bool full = (c + 8 <= p.cout);
  const int cnt = full ? 8 : (p.cout - c);
  if (add_bias && p.bias) {
#pragma unroll
    for (int i = 0; i < 8; ++i) if (i < cnt) v[i] += p.bias[c + i];
  }
  if (p.rowbias) {
    const bf16* rb = p.rowbias + (long)(*p.rowbias_idx) * p.rowbias_ld + c;
#pragma unroll
    for (int i = 0; i < 8; ++i) if (i < cnt) v[i] = (float)(bf16)v[i] + (float)rb[i];
  }
  if (p.resid) {
    const bf16* r = p.resid + m * p.ldr + c;
    if (full) {
      float rf[8];
      load8(r, rf);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + rf[i];
    } else {
      for (int i = 0; i < cnt; ++i) v[i] = (float)(bf16)v[i] + (float)r[i];
    }
  }
  if (p.act == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.0f);
  }
  if (p.mask) {
    const bf16* mk = p.mask + m * p.ldmask + c;
    if (full) {
      float mf[8];
      load8(mk, mf);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = mf[i] > 0.0f ? v[i] : 0.0f;
    } else {
      for (int i = 0; i < cnt; ++i) v[i] = (float)mk[i] > 0.0f ? v[i] : 0.0f;
    }
  }
  bf16* out = p.y + m * p.ldy + c;
  if (full) {
    store8(out, v);
  } else {
    for (int i = 0; i < cnt; ++i) out[i] = (bf16)v[i];
  }
}

// ---- epilogue operands loaded ahead.  Loaded where epilogue_store uses them, the column bias, then the row-bias /
// residual / mask vectors are each a dependent memory round trip at the end of the tile (after the staging barrier);
// loaded at kernel start (or before the staging barrier where the registers are scarce) they land under the main
// loop.  RMAX = the lane's 16-B output rows (lane + 64 r of the wave's WM x WN / 8 row-vectors; GPR divides 64, so a
// lane keeps one 8-channel column group).
// kEpiEarly: load them at kernel start.  Off: holding them across the main loop cost 20-90 VGPRs in most im2col
// instantiations (128 x 128 x 32: 140 -> 228, 128 x 64 x 64: 144 -> 188) and a wave per SIMD of occupancy, which the
// runtime A/B (DC_HALO_DIAG=256, same binary) could not show: C3 conv launches +21 % (profiles/r04z).  The epilogue
// then loads every operand after the main loop (the round-3 placement).  Build-time switch, left out of the default
// build (-DDC_EPI_EARLY=1 compiles the early placement in; DC_HALO_DIAG=256 then selects it per launch).
#ifndef DC_EPI_EARLY
#define DC_EPI_EARLY 0
#endif
constexpr bool kEpiEarly = DC_EPI_EARLY != 0;
template <int NJ, int RMAX>
struct EpiPre {
  float cv[NJ];        // per-column bias (GNM 3: csum)
  float cv2[NJ];       // GNM 3: cbias
  bf16x8 rb;           // row bias (per-step table row) of the lane's 8 columns
  bf16x8 res[RMAX], msk[RMAX];
  long mrow[RMAX];     // output pixel of each row-vector (-1: none)
};
template <int GNM, int NJ, int RMAX>
__device__ __forceinline__ void epi_cols(const ConvGemmParams& p, int c0, EpiPre<NJ, RMAX>& e) {
  // c0 = the lane's first column (n0 + wn WN + lane % 16); column j = c0 + 16 j
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = c0 + j * 16;
    if constexpr (GNM == 3) {
      e.cv[j] = c < p.cout ? p.ln_csum[c] : 0.0f;
      e.cv2[j] = c < p.cout ? p.ln_cbias[c] : 0.0f;
    } else {
      e.cv[j] = (p.bias && c < p.cout) ? p.bias[c] : 0.0f;
    }
  }
}
template <int WM, int GPR, int NJ, int RMAX>
__device__ __forceinline__ void epi_rows(const ConvGemmParams& p, long mw, int c, long M, int lane,
                                         EpiPre<NJ, RMAX>& e) {
  // mw = the wave's first output row, c = the lane's 8-channel group (n0 + wn WN + (lane % GPR) 8)
  const bool full = c + 8 <= p.cout;
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    const int g = lane + 64 * r;
    const long m = mw + g / GPR;
    e.mrow[r] = (g < WM * GPR && m < M && c < p.cout) ? conv_pix(p, m) : -1;
    if (e.mrow[r] >= 0 && full) {
      if (p.resid) e.res[r] = *reinterpret_cast<const bf16x8*>(p.resid + e.mrow[r] * p.ldr + c);
      if (p.mask) e.msk[r] = *reinterpret_cast<const bf16x8*>(p.mask + e.mrow[r] * p.ldmask + c);
    }
  }
  if (p.rowbias && full) e.rb = *reinterpret_cast<const bf16x8*>(p.rowbias + (long)(*p.rowbias_idx) * p.rowbias_ld + c);
}
// epilogue_store with the row-vector's preloaded operands (partial vectors, cout % 8 != 0, load as before)
template <int NJ, int RMAX>
__device__ __forceinline__ void epilogue_store_pre(const ConvGemmParams& p, const EpiPre<NJ, RMAX>& e, int r, int c,
                                                   float* v) {
  const long m = e.mrow[r];
  if (c + 8 > p.cout) {
    epilogue_store(p, m, c, v, false);
    return;
  }
  if (p.rowbias) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + (float)e.rb[i];
  }
  if (p.resid) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + (float)e.res[r][i];
  }
  if (p.act == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.0f);
  }
  if (p.mask) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)e.msk[r][i] > 0.0f ? v[i] : 0.0f;
  }
  store8(p.y + m * p.ldy + c, v);
}

// ---- GroupNorm statistics fused into the epilogue (include/dcamd.h dc_gn_fuse; the host guarantees cout % 8 == 0,
// no row list, no GEGLU).  The epilogue's 16-B row loop gives each lane one 8-channel column group cg = lane % GPR
// (GPR divides 64) over rows g / GPR: the lane sums its channels over its rows, the sums are reduced over the lanes
// of the same column group, and one lane per column group adds each group's share (runs of its 8 channels) to the
// accumulators.  A wave whose rows straddle two frames (linears over nb * T rows, T not a multiple of the wave's
// rows) adds per row instead.

// the final values of a full 8-channel vector (epilogue_store without the store), rounded to the stored bf16
__device__ __forceinline__ void epilogue_values8(const ConvGemmParams& p, long m, int c, float* v) {
  if (p.rowbias) {
    const bf16* rb = p.rowbias + (long)(*p.rowbias_idx) * p.rowbias_ld + c;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + (float)rb[i];
  }
  if (p.resid) {
    float rf[8];
    load8(p.resid + m * p.ldr + c, rf);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + rf[i];
  }
  if (p.act == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.0f);
  }
  if (p.mask) {
    float mf[8];
    load8(p.mask + m * p.ldmask + c, mf);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = mf[i] > 0.0f ? v[i] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i];
}

// add channel sums (s, q)[8] of output channels c .. c + 7, frame f, to target t: one add per group run
__device__ __forceinline__ void gn_add_channels(const GnTargetP& t, int f, int c, const float* s, const float* q) {
  unsigned long long* base = t.acc + ((blockIdx.x + blockIdx.y) & (kGnReplicas - 1)) * t.rstride +
                             (long)f * t.groups * kGnPair;
  int g = (c + t.coff) / t.cpg;
  int left = (g + 1) * t.cpg - (c + t.coff);   // channels of group g from channel c on
  float a = 0.0f, b = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a += s[i];
    b += q[i];
    if (--left == 0 || i == 7) {
      unsigned long long* w = base + (long)g * kGnPair;
      gn_acc_add(w, a);
      gn_acc_add(w + kGnWords, b);
      a = b = 0.0f;
      ++g;
      left = t.cpg;
    }
  }
}

// Rows of one wave.  pix_of(row) = output pixel of wave row `row` (or -1); fa / fb = frames of the block's first
// and last valid pixel (block-uniform: a block in one frame reduces its sums in LDS and adds once per group, a
// block across frames adds per lane and row); es / lde: the wave's bf16 staging tile; wave (wm, wn) of a WGM x WGN
// layout covering BN output channels from n0; LDS: the kernel's LDS bytes (the reduction needs 16 KB + 8 BN).
// Every wave of the block calls this (the one-frame form has barriers).  The output values are kept in registers
// (bf16) until the accumulator adds are issued, so that the adds' memory-side round trip overlaps the stores'.
template <int GNM, int WM, int WN, int BN, int WGM, int LDS, typename PixFn>
__device__ __forceinline__ void gn_epilogue_rows(const ConvGemmParams& p, char* smem, const bf16* es, int lde, int n0,
                                                 int wm, int wn, int lane, int fa, int fb, PixFn pix_of) {
  constexpr int GPR = WN / 8;
  constexpr int RMAX = (WM * GPR + 63) / 64;   // rows per lane
  static_assert(LDS >= 64 * 4 * 16 * 4 + 2 * BN * 4, "GroupNorm-statistics reduction LDS");
  static_assert(64 % GPR == 0, "a lane's rows share one 8-channel column group");
  if (p.diag & 64) return;   // experiments only: no epilogue at all
  const GnFuseP& G = p.gn;
  const GnTargetP& t0 = G.t[0];
  const int cg = lane % GPR;
  const int c = n0 + wn * WN + cg * 8;
  const bool cok = c < p.cout;
  const bool uni = fa == fb;
  float s[8], q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = q[i] = 0.0f;
  // backward: the lane's channel constants and its channels' (mean, rstd) in the current frame
  float ga[8], be[8], mu[8], rs[8];
  int fcur = -1;
  if (GNM == 2 && cok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ga[i] = G.gamma[c + i];
      be[i] = G.beta[c + i];
    }
  }
  bf16x8 keep[RMAX];
  long mrow[RMAX];
  // the global operands of the lane's rows in one batch ahead of the staging reads and the arithmetic (the row bias,
  // residual and -- backward -- the GroupNorm input x and the frame's (mean, rstd)); loaded per row where they are
  // used, each was a dependent memory round trip behind the staging reads or the frame test
  bf16x8 rres[RMAX], rx[GNM == 2 ? RMAX : 1], rbias;
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    const int g = lane + 64 * r;
    mrow[r] = (g < WM * GPR && cok) ? pix_of(g / GPR) : -1;
    const long m = mrow[r];
    if (m < 0) continue;
    if (p.resid) rres[r] = *reinterpret_cast<const bf16x8*>(p.resid + m * p.ldr + c);
    if constexpr (GNM == 2)
      rx[r] = c < G.c1 ? *reinterpret_cast<const bf16x8*>(G.x + m * G.ldx + c)
                       : *reinterpret_cast<const bf16x8*>(G.x2 + m * G.ldx2 + (c - G.c1));
  }
  if (p.rowbias && cok) rbias = *reinterpret_cast<const bf16x8*>(p.rowbias + (long)(*p.rowbias_idx) * p.rowbias_ld + c);
  auto load_stats = [&](int f) {
    const float* st = G.stats + (long)f * t0.groups * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int gi = (c + i) / t0.cpg;
      mu[i] = st[gi * 2];
      rs[i] = st[gi * 2 + 1];
    }
    fcur = f;
  };
  if (GNM == 2 && uni && cok) load_stats(fa);
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    const int row = (lane + 64 * r) / GPR;
    const long m = mrow[r];
    if (m < 0) continue;
    float v[8];
    load8(es + row * lde + cg * 8, v);
    // epilogue_values8 with the preloaded operands
    if (p.rowbias) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + (float)rbias[i];
    }
    if (p.resid) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i] + (float)rres[r][i];
    }
    if (p.act == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.0f);
    }
    if (p.mask) {
      float mf[8];
      load8(p.mask + m * p.ldmask + c, mf);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = mf[i] > 0.0f ? v[i] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)(bf16)v[i];
    const int f = uni ? fa : (int)fast_div((unsigned)m, t0.hw_mul, t0.hw_shr);
    if constexpr (GNM == 2) {
      if (f != fcur) load_stats(f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = ((float)rx[r][i] - mu[i]) * rs[i];
        float dd = v[i];
        if (G.silu) {
          const float yv = (float)(bf16)(xh * ga[i] + be[i]);
          dd = (float)(bf16)(dd * silu_grad(yv));
        }
        const float gd = dd * ga[i];
        s[i] += gd;
        q[i] += gd * xh;
        v[i] = dd;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s[i] += v[i];
        q[i] += v[i] * v[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) keep[r][i] = (bf16)v[i];
    if (!uni) {
      for (int k = 0; k < G.nt; ++k) gn_add_channels(G.t[k], f, c, s, q);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = q[i] = 0.0f;
    }
  }
  if (uni && !(p.diag & 16)) {
    // one frame: lane sums -> LDS [wave][lane][16]; thread ch < BN sums its channel's WGM x 64 / GPR entries
    // (fixed order) -> colsum; one thread per group of the tile's channels adds the group's sums
    float* red = reinterpret_cast<float*>(smem);
    float* col = red + 4 * 64 * 16;
    const int wid = threadIdx.x >> 6;
    __syncthreads();   // every wave is done with its staging tile
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(wid * 64 + lane) * 16 + i] = s[i];
      red[(wid * 64 + lane) * 16 + 8 + i] = q[i];
    }
    __syncthreads();
    const int tid = threadIdx.x;
    if (tid < BN) {
      const int cwn = tid / WN, cw = tid - cwn * WN, ccg = cw >> 3, ci = cw & 7;
      float a = 0.0f, b = 0.0f;
#pragma unroll
      for (int w = 0; w < WGM; ++w) {
        const int wv = w * (4 / WGM) + cwn;   // wave id of (wm = w, wn = cwn): wid = wm * WGN + wn
#pragma unroll
        for (int j = 0; j < 64 / GPR; ++j) {
          const float* e = red + (wv * 64 + ccg + GPR * j) * 16;
          a += e[ci];
          b += e[8 + ci];
        }
      }
      col[tid] = a;
      col[BN + tid] = b;
    }
    __syncthreads();
    const int cend = min(n0 + BN, p.cout);
    if (!(p.diag & 8)) {
      for (int k = 0; k < G.nt; ++k) {
        const GnTargetP& t = G.t[k];
        const int g = (n0 + t.coff) / t.cpg + tid;
        const int lo = max(g * t.cpg - t.coff, n0), hi = min((g + 1) * t.cpg - t.coff, cend);
        if (lo < hi) {
          float a = 0.0f, b = 0.0f;
          for (int ch = lo; ch < hi; ++ch) {
            a += col[ch - n0];
            b += col[BN + ch - n0];
          }
          unsigned long long* w = t.acc + ((blockIdx.x + blockIdx.y) & (kGnReplicas - 1)) * t.rstride +
                                  ((long)fa * t.groups + g) * kGnPair;
          gn_acc_add(w, a);
          gn_acc_add(w + kGnWords, b);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RMAX; ++r)
    if (mrow[r] >= 0) *reinterpret_cast<bf16x8*>(p.y + mrow[r] * p.ldy + c) = keep[r];
}

// ---- fused GroupNorm statistics for the block-staged epilogues (the skinny kernels and their split-K reduce kernel):
// the block's store loop visits (row, 8-channel column group) pairs g = tid, tid + 256, ... so a thread keeps one
// column group (GPR = BN / 8 divides 256).  add() takes a row's final values (epilogue_values8) and, for GNM 2, turns
// them into dy' (stored in their place) as gn_epilogue_rows does; the running sums belong to one frame and are added
// per thread when the frame changes (row runs across frames: batched linears).  finish(): a block whose rows lie in
// one frame folds its threads' sums in LDS (fixed order) and adds once per group; otherwise each thread adds its own.
template <int GNM, int GPR>
struct GnTileSums {
  float s[8], q[8];
  float ga[8], be[8], mu[8], rs[8];
  int fcur;   // frame of the running sums (-1: none yet)
  int fst;    // frame of the loaded (mean, rstd) (GNM 2)
  int c;      // the thread's first channel (-1: no column group in range)

  __device__ __forceinline__ void init(const ConvGemmParams& p, int c0) {
    c = c0 < p.cout ? c0 : -1;
    fcur = fst = -1;
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = q[i] = 0.0f;
    if (GNM == 2 && c >= 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ga[i] = p.gn.gamma[c + i];
        be[i] = p.gn.beta[c + i];
      }
    }
  }
  __device__ __forceinline__ void flush(const ConvGemmParams& p) {
    if (fcur < 0) return;
    if (!(p.diag & 8))
      for (int k = 0; k < p.gn.nt; ++k) gn_add_channels(p.gn.t[k], fcur, c, s, q);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = q[i] = 0.0f;
    fcur = -1;
  }
  // row m (frame f) of the thread's column group: v = the stored values on return
  __device__ __forceinline__ void add(const ConvGemmParams& p, long m, int f, float* v) {
    if (f != fcur) {
      flush(p);
      fcur = f;
    }
    if constexpr (GNM == 2) {
      const GnFuseP& G = p.gn;
      if (f != fst) {
        const float* st = G.stats + (long)f * G.t[0].groups * 2;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int gi = (c + i) / G.t[0].cpg;
          mu[i] = st[gi * 2];
          rs[i] = st[gi * 2 + 1];
        }
        fst = f;
      }
      float xf[8];
      if (c < G.c1) load8(G.x + m * G.ldx + c, xf);
      else load8(G.x2 + m * G.ldx2 + (c - G.c1), xf);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (xf[i] - mu[i]) * rs[i];
        float dd = v[i];
        if (G.silu) {
          const float yv = (float)(bf16)(xh * ga[i] + be[i]);
          dd = (float)(bf16)(dd * silu_grad(yv));
        }
        const float gd = dd * ga[i];
        s[i] += gd;
        q[i] += gd * xh;
        v[i] = dd;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s[i] += v[i];
        q[i] += v[i] * v[i];
      }
    }
  }
  // every thread of the block; uni: all the block's rows are in frame fa.  red: >= (256 * 16 + 2 * BN) floats of LDS
  // that no thread reads any more (the barrier first)
  template <int BN>
  __device__ __forceinline__ void finish(const ConvGemmParams& p, float* red, int n0, bool uni, int fa) {
    if (!uni) {
      if (c >= 0) flush(p);
      return;
    }
    const int tid = threadIdx.x;
    float* col = red + 256 * 16;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[tid * 16 + i] = s[i];
      red[tid * 16 + 8 + i] = q[i];
    }
    __syncthreads();
    if (tid < BN) {
      const int ccg = tid >> 3, ci = tid & 7;
      float a = 0.0f, b = 0.0f;
#pragma unroll
      for (int j = 0; j < 256 / GPR; ++j) {
        a += red[(ccg + GPR * j) * 16 + ci];
        b += red[(ccg + GPR * j) * 16 + 8 + ci];
      }
      col[tid] = a;
      col[BN + tid] = b;
    }
    __syncthreads();
    if (p.diag & 8) return;
    const int cend = min(n0 + BN, p.cout);
    for (int k = 0; k < p.gn.nt; ++k) {
      const GnTargetP& t = p.gn.t[k];
      const int g = (n0 + t.coff) / t.cpg + tid;
      const int lo = max(g * t.cpg - t.coff, n0), hi = min((g + 1) * t.cpg - t.coff, cend);
      if (lo < hi) {
        float a = 0.0f, b = 0.0f;
        for (int ch = lo; ch < hi; ++ch) {
          a += col[ch - n0];
          b += col[BN + ch - n0];
        }
        unsigned long long* w = t.acc + ((blockIdx.x + blockIdx.y) & (kGnReplicas - 1)) * t.rstride +
                                ((long)fa * t.groups + g) * kGnPair;
        gn_acc_add(w, a);
        gn_acc_add(w + kGnWords, b);
      }
    }
  }
};

// -DDC_DEBUG_LDS (debug builds only, tools/debug_lds.sh): every LDS-DMA wave-instruction's 1 KiB destination and
// every epilogue staging row is asserted inside the block's static LDS allocation
#ifdef DC_DEBUG_LDS
#define DC_LDS_ASSERT(off, bytes, limit)                                                                  \
  do {                                                                                                    \
    const int dc_o_ = (off);                                                                              \
    if (dc_o_ < 0 || dc_o_ + (bytes) > (limit)) {                                                         \
      printf("DC_DEBUG_LDS %s:%d block %d thread %d: LDS offset %d + %d outside %d\n", __FILE__, __LINE__, \
             (int)blockIdx.x, (int)threadIdx.x, dc_o_, (int)(bytes), (int)(limit));                       \
      __builtin_trap();                                                                                   \
    }                                                                                                     \
  } while (0)
#else
#define DC_LDS_ASSERT(off, bytes, limit) ((void)0)
#endif

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `ahead` k-chunks (L pieces each) remain in flight
template <int L, int S>
__device__ __forceinline__ void wait_chunks(int ahead) {
  static_assert(S >= 2 && S <= 8, "stages");
  switch (ahead) {
    case 0: vm_wait<0>(); break;
    case 1: vm_wait<(S > 2 ? L : 0)>(); break;
    case 2: vm_wait<(S > 3 ? 2 * L : 0)>(); break;
    case 3: vm_wait<(S > 4 ? 3 * L : 0)>(); break;
    case 4: vm_wait<(S > 5 ? 4 * L : 0)>(); break;
    case 5: vm_wait<(S > 6 ? 5 * L : 0)>(); break;
    default: vm_wait<(S > 7 ? 6 * L : 0)>(); break;
  }
}

// LDS bytes: S ring stages of (BM + BN) rows x BK bf16, reused by the per-wave bf16 epilogue tile
template <int BM, int BN, int BK, int S>
struct Cfg {
  static constexpr int RB = BK * 2;                                     // bytes per tile row per stage
  static constexpr int STAGE = (BM + BN) * RB;
  static constexpr int EPI = 4 * (BM / 2) * (BN / 2 + 8) * 2;          // 4 waves x [WM][WN+8] bf16
  static constexpr int LDS = (S * STAGE > EPI) ? S * STAGE : EPI;
};

// XOR swizzle of the 16-B chunk index within a tile row, chosen so that the ds_read_b128 fragment
// reads (16 consecutive rows x 4 chunks per instruction, lanes grouped 0-3/12-15/20-27 ... by the
// LDS crossbar) are conflict-free: BK=64 rows are 8 chunks (128 B) wide, BK=32 rows 4 chunks.
template <int BK>
__device__ __forceinline__ int swz(int row) {
  if constexpr (BK == 64) return row & 7;
  else return ((row >> 3) & 1) << 1;
}

// Mainloop of one (tile, k-range) segment: gathers A / W chunks [kc_begin, kc_end) through the LDS ring
// and accumulates into acc (zeroed here).  Ends with every LDS-DMA landed; the ring is still being read
// by other waves until the caller's next barrier.
template <int BM, int BN, int BK, int S, bool SMALLC>
__device__ __forceinline__ void tile_pass(const ConvGemmParams& p, char* smem, long m0, int n0, int kc_begin,
                                          int kc_end, f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int CPR = BK / 8;            // 16-B chunks per tile row
  constexpr int RPI = 256 / CPR;         // tile rows covered by one block-wide LDS-DMA instruction
  constexpr int AP = BM / RPI;           // A pieces (16 B) per thread per k-chunk
  constexpr int BP = BN / RPI;
  constexpr int L = AP + BP;             // LDS-DMA instructions per thread per k-chunk
  constexpr int KS = BK / 32;            // MFMA k-steps per chunk
  constexpr int RB = Cfg<BM, BN, BK, S>::RB;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NJ = WN / 16;
  constexpr int STAGE = Cfg<BM, BN, BK, S>::STAGE;
  static_assert(AP >= 1 && BP >= 1, "tile too small for the block-wide DMA");

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // wave index as a scalar: the LDS-DMA destination (M0) of every piece is then SALU arithmetic
  const int wid_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned hwo = (unsigned)(p.hout * p.wout);
  const long M = conv_rows(p);
  const int nkc = max(0, kc_end - kc_begin);

  // per-thread A-row gather tables (piece j covers tile row tid/CPR + RPI j, chunk slot tid%CPR):
  // source pixel = ypix[ky] + xpix[kx] for every mode (direct / upsample / transposed), valid-tap bitmask
  const int slot = tid % CPR;
  struct RowTab {
    int y0, y1, y2, x0, x1, x2;
  };
  RowTab rt[AP];
  int a_sw[AP];
  unsigned vmask[AP];
  int pn[AP], poy[AP], pox[AP];  // !SMALLC: output pixel (frame, y, x) of each piece's row; pn < 0 past M
#pragma unroll
  for (int j = 0; j < AP; ++j) {
    const int row = tid / CPR + RPI * j;
    a_sw[j] = slot ^ swz<BK>(row);  // logical 16-B chunk this lane fetches (XOR swizzle via the source)
    const long m = m0 + row;
    vmask[j] = 0u;
    if constexpr (!SMALLC) {
      const bool in = m < M;
      const unsigned mp = in ? (unsigned)conv_pix(p, m) : 0u;
      const unsigned n = fast_div(mp, p.hw_mul, p.hw_shr);
      const unsigned rem = mp - n * hwo;
      const unsigned oy = fast_div(rem, p.w_mul, p.w_shr);
      pn[j] = in ? (int)n : -1;
      poy[j] = (int)oy;
      pox[j] = (int)(rem - oy * (unsigned)p.wout);
      continue;
    }
    int yp[3] = {0, 0, 0}, xp[3] = {0, 0, 0};
    if (m < M) {
      const unsigned mp = (unsigned)conv_pix(p, m);
      const int n = (int)fast_div(mp, p.hw_mul, p.hw_shr);
      const int rem = (int)(mp - (unsigned)n * hwo);
      const int oy = (int)fast_div((unsigned)rem, p.w_mul, p.w_shr), ox = rem - oy * p.wout;
      unsigned yv = 0u, xv = 0u;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        int iy, ix;
        bool oky, okx;
        if (p.mode == 0) {
          iy = oy * p.stride - p.pad + t;
          ix = ox * p.stride - p.pad + t;
          oky = iy >= 0 && iy < p.hin;
          okx = ix >= 0 && ix < p.win;
        } else if (p.mode == 1) {
          const int vy = oy - p.pad + t, vx = ox - p.pad + t;
          oky = vy >= 0 && vy < p.hout;
          okx = vx >= 0 && vx < p.wout;
          iy = oky ? (int)fast_div((unsigned)(vy * p.hin), p.h_mul, p.h_shr) : 0;
          ix = okx ? (int)fast_div((unsigned)(vx * p.win), p.w_mul, p.w_shr) : 0;
        } else {
          const int ty = oy - 1 + t, tx = ox - 1 + t;
          oky = ty >= 0 && !(ty & 1) && (ty >> 1) < p.hin;
          okx = tx >= 0 && !(tx & 1) && (tx >> 1) < p.win;
          iy = ty >> 1;
          ix = tx >> 1;
        }
        oky = oky && t < p.kh;
        okx = okx && t < p.kw;
        yp[t] = oky ? (n * p.hin + iy) * p.win : 0;
        xp[t] = okx ? ix : 0;
        yv |= (oky ? 1u : 0u) << t;
        xv |= (okx ? 1u : 0u) << t;
      }
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx)
          if (((yv >> ty) & 1u) && ((xv >> tx) & 1u)) vmask[j] |= 1u << (ty * p.kw + tx);
    }
    rt[j] = RowTab{yp[0], yp[1], yp[2], xp[0], xp[1], xp[2]};
  }
  const int cch = SMALLC ? 1 : (p.cin / BK);
  const bf16* zero = (const bf16*)g_zero_line;

  // ---- producer.  !SMALLC: buffer_load ... lds with a per-lane 32-bit voffset that is fixed for a
  // whole tap (recomputed only when the tap changes) and the channel offset of the chunk in the
  // scalar soffset, so a chunk costs no address VALU; padding / tails read out of range (offset
  // >= 2 GiB, zero-filled by the buffer unit).  SMALLC (cin % 64 != 0, first layers) keeps a
  // per-piece LDS-DMA gather from the zero line.
  constexpr int kOOB = (int)0x80000000u;
  const __amdgpu_buffer_rsrc_t ra = buf_rsrc(p.x);
  const __amdgpu_buffer_rsrc_t ra2 = buf_rsrc(p.x2);
  const __amdgpu_buffer_rsrc_t rb = buf_rsrc(p.w);
  int a_off[AP], a_off2[AP], b_off[BP];
#pragma unroll
  for (int j = 0; j < BP; ++j) {
    const int row = tid / CPR + RPI * j;
    const int co = n0 + row;
    b_off[j] = co < p.cout ? (co * p.ktot + (slot ^ swz<BK>(row)) * 8) * 2 : kOOB;
  }
  const bool two_src = p.c1 < p.cin;
  // voffsets of the current tap, recomputed from the pixel coordinates (9 times per conv at most)
  auto set_tap = [&](int tap) __attribute__((always_inline)) {
    const int ty = p.kw == 3 ? tap / 3 : 0, tx = p.kw == 3 ? tap - (tap / 3) * 3 : 0;
#pragma unroll
    for (int j = 0; j < AP; ++j) {
      int iy, ix;
      bool ok;
      if (p.mode == 0) {
        iy = poy[j] * p.stride - p.pad + ty;
        ix = pox[j] * p.stride - p.pad + tx;
        ok = iy >= 0 && iy < p.hin && ix >= 0 && ix < p.win;
      } else if (p.mode == 1) {
        const int vy = poy[j] - p.pad + ty, vx = pox[j] - p.pad + tx;
        ok = vy >= 0 && vy < p.hout && vx >= 0 && vx < p.wout;
        iy = ok ? (int)fast_div((unsigned)(vy * p.hin), p.h_mul, p.h_shr) : 0;
        ix = ok ? (int)fast_div((unsigned)(vx * p.win), p.w_mul, p.w_shr) : 0;
      } else {
        const int yy = poy[j] - 1 + ty, xx = pox[j] - 1 + tx;
        ok = yy >= 0 && !(yy & 1) && (yy >> 1) < p.hin && xx >= 0 && !(xx & 1) && (xx >> 1) < p.win;
        iy = yy >> 1;
        ix = xx >> 1;
      }
      ok = ok && pn[j] >= 0;
      const int pix = (pn[j] * p.hin + iy) * p.win + ix;
      a_off[j] = ok ? (pix * p.ldx + a_sw[j] * 8) * 2 : kOOB;
      if (two_src) a_off2[j] = ok ? (pix * p.ldx2 + a_sw[j] * 8) * 2 : kOOB;
    }
  };
  // issue cursor: next chunk's tap and channel offset (one division at the start of the range)
  // (readfirstlane: the integer division runs on the VALU, and a VGPR soffset / branch condition would
  // be waterfalled)
  int q_k = kc_begin;
  int q_tap = SMALLC ? 0 : __builtin_amdgcn_readfirstlane(kc_begin / cch);
  int q_c = SMALLC ? 0 : __builtin_amdgcn_readfirstlane((kc_begin - q_tap * cch) * BK);
  if (!SMALLC && nkc > 0) set_tap(q_tap);

  auto issue = [&](int stage) __attribute__((always_inline)) {
    DC_LDS char* sbase = (DC_LDS char*)smem + stage * STAGE;
#ifdef DC_DEBUG_LDS
    for (int j = 0; j < AP; ++j)
      DC_LDS_ASSERT(stage * STAGE + (wid_s * 64 + 256 * j) * 16, 1024, (Cfg<BM, BN, BK, S>::LDS));
    for (int j = 0; j < BP; ++j)
      DC_LDS_ASSERT(stage * STAGE + BM * RB + (wid_s * 64 + 256 * j) * 16, 1024, (Cfg<BM, BN, BK, S>::LDS));
#endif
    if (!SMALLC) {
      if (q_c >= p.c1) {  // uniform: the chunk comes from the second concat source
#pragma unroll
        for (int j = 0; j < AP; ++j)
          buf_load_lds16(ra2, sbase + (wid_s * 64 + 256 * j) * 16, a_off2[j], (q_c - p.c1) * 2);
      } else {
#pragma unroll
        for (int j = 0; j < AP; ++j)
          buf_load_lds16(ra, sbase + (wid_s * 64 + 256 * j) * 16, a_off[j], q_c * 2);
      }
    } else {
#pragma unroll
      for (int j = 0; j < AP; ++j) {
        const int k = q_k * BK + a_sw[j] * 8;
        const int tap = k / p.cin;
        const int c = k - tap * p.cin;
        const int ky = tap / p.kw, kx = tap - (tap / p.kw) * p.kw;
        const bool ok = tap < p.kh * p.kw && ((vmask[j] >> tap) & 1u);
        const int pix = (ky == 0 ? rt[j].y0 : (ky == 1 ? rt[j].y1 : rt[j].y2)) +
                        (kx == 0 ? rt[j].x0 : (kx == 1 ? rt[j].x1 : rt[j].x2));
        const bf16* src = ok ? p.x + (long)pix * p.ldx + c : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, sbase + (wid_s * 64 + 256 * j) * 16, 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BP; ++j)
      buf_load_lds16(rb, sbase + BM * RB + (wid_s * 64 + 256 * j) * 16, b_off[j], q_k * BK * 2);
    ++q_k;
    if (!SMALLC) {
      q_c += BK;
      if (q_c == p.cin) {
        q_c = 0;
        ++q_tap;
        if (q_k < kc_end) set_tap(q_tap);
      }
    }
  };

#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int s = 0; s < S - 1 && s < nkc; ++s) issue(s);
  for (int i = 0; i < nkc; ++i) {
    // steady state: S - 2 younger chunks stay in flight (one compare instead of the wait cascade)
    if (i + S - 2 < nkc) vm_wait<(S - 2) * L>();
    else wait_chunks<L, S>(nkc - 1 - i);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (i + S - 1 < nkc) issue((i + S - 1) % S);
    const char* sa = smem + (i % S) * STAGE;
    const char* sb = sa + BM * RB;
    bf16x8 af[KS][MI], bfr[KS][NJ];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int ii = 0; ii < MI; ++ii) {
        const int row = wm * WM + ii * 16 + (lane & 15);
        af[ks][ii] = *reinterpret_cast<const bf16x8*>(sa + row * RB + ((chunk ^ swz<BK>(row)) << 4));
      }
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj) {
        const int row = wn * WN + jj * 16 + (lane & 15);
        bfr[ks][jj] = *reinterpret_cast<const bf16x8*>(sb + row * RB + ((chunk ^ swz<BK>(row)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj)
          acc[ii][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][ii], bfr[ks][jj], acc[ii][jj], 0, 0, 0);
    // keep every fragment read of the chunk ahead of its MFMAs (the default schedule interleaves
    // read -> lgkmcnt(0) -> 2 MFMAs, exposing the LDS latency once per fragment)
    __builtin_amdgcn_sched_group_barrier(0x100, KS * (MI + NJ), 0);
    __builtin_amdgcn_sched_group_barrier(0x008, KS * MI * NJ, 0);
  }
  vm_wait<0>();
}

// Partial-sum hand-off of a tile computed in `narrive` k-segments (deterministic: the tile's
// last-arriving block sums every segment's partial in segment order).  Partials go out in the
// accumulator-native layout [slot][wave][i][j][lane] as 16-B sc1 stores; one lane per block then bumps
// the tile's counter (agent-scope atomic) after every wave's vmcnt(0); the block that arrives last reads
// all partials back with sc1 loads (MI355X_MICROARCH.md hand-off table, row 1), leaves their sum in acc
// and returns true (the caller then runs the epilogue).  slot_of(i) = slab slot of segment i.
// (MI x NJ 16x16 accumulators per wave, 4 waves: any wave layout of the tile)
template <int MI, int NJ, typename SlotFn>
__device__ __forceinline__ bool tile_handoff_g(const ConvGemmParams& p, char* smem, int tile, int my_slot, int narrive,
                                               SlotFn slot_of, f32x4 (&acc)[MI][NJ]) {
  constexpr int WAVE_F = MI * NJ * 256;
  constexpr int TILE_F = 4 * WAVE_F;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const __amdgpu_buffer_rsrc_t rs = ws_rsrc(p.ws);
  const long slab = (long)my_slot * TILE_F + wid * WAVE_F + lane * 4;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) store_sc1_x4(rs, slab + (i * NJ + j) * 256, acc[i][j]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the flag lives in the (now idle) ring: a second __shared__ object would make the compiler's
  // waitcnt pass treat every LDS-DMA as aliasing the main loop's ds_reads (vmcnt(0) per chunk)
  int* s_last = reinterpret_cast<int*>(smem);
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = old == narrive - 1;
  }
  __syncthreads();
  if (!*s_last) return false;
  // every segment's partial (this block's own included) is read back in segment order
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one accumulator row i at a time, GS segments' loads in flight per round (8 x 16 B per lane: the
  // register peak stays that of the main loop's fragments), added in segment order -- one round trip
  // per GS segments instead of per segment
  constexpr int GS = NJ >= 8 ? 1 : 8 / NJ;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    for (int sp0 = 0; sp0 < narrive; sp0 += GS) {
      f32x4 part[GS][NJ];
#pragma unroll
      for (int g = 0; g < GS; ++g) {
        if (sp0 + g < narrive) {
          const long src = (long)slot_of(sp0 + g) * TILE_F + wid * WAVE_F + lane * 4;
#pragma unroll
          for (int j = 0; j < NJ; ++j) part[g][j] = load_sc1_x4(rs, src + (i * NJ + j) * 256);
        }
      }
#pragma unroll
      for (int g = 0; g < GS; ++g) {
        if (sp0 + g < narrive) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] += part[g][j];
        }
      }
    }
  }
  if (tid == 0) p.counters[tile] = 0;  // ready for the next launch (ordered by the kernel boundary)
  return true;
}
template <int BM, int BN, typename SlotFn>
__device__ __forceinline__ bool tile_handoff(const ConvGemmParams& p, char* smem, int tile, int my_slot, int narrive,
                                             SlotFn slot_of, f32x4 (&acc)[BM / 32][BN / 32]) {
  return tile_handoff_g<BM / 32, BN / 32>(p, smem, tile, my_slot, narrive, slot_of, acc);
}

// the preloaded epilogue operands of a BM x BN tile (4 waves, 2 x 2)
template <int BM, int BN>
struct TileEpi {
  static constexpr int WM = BM / 2, WN = BN / 2, NJ = WN / 16, GPR = WN / 8;
  static constexpr int RMAX = (WM * GPR + 63) / 64;
  // a lane keeps one 8-channel column group only where GPR divides 64 (not the 320-wide tiles): else no row preload
  static constexpr bool kRows = 64 % GPR == 0;
  static constexpr bool kEarly = kRows && RMAX <= 4;   // row operands loaded at kernel start (else before the staging)
  using Pre = EpiPre<NJ, RMAX>;
};
template <int BM, int BN, int GNM>
__device__ __forceinline__ void tile_epi_load(const ConvGemmParams& p, long m0, int n0, bool rows,
                                              typename TileEpi<BM, BN>::Pre& e) {
  using TE = TileEpi<BM, BN>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  if (!rows) epi_cols<GNM>(p, n0 + wn * TE::WN + (lane & 15), e);
  if (rows && TE::kRows && GNM != 1 && GNM != 2 && !p.geglu)
    epi_rows<TE::WM, TE::GPR>(p, m0 + wm * TE::WM, n0 + wn * TE::WN + (lane % TE::GPR) * 8, conv_rows(p), lane, e);
}

// epilogue: bias in fp32, round to bf16 into a per-wave LDS tile, then 16-B coalesced rows
template <int BM, int BN, int GNM, int LDSB>
__device__ __forceinline__ void tile_epilogue(const ConvGemmParams& p, char* smem, long m0, int n0,
                                              const f32x4 (&acc)[BM / 32][BN / 32], typename TileEpi<BM, BN>::Pre& pre) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NJ = WN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const long M = conv_rows(p);
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
  if (kEpiEarly && (!TileEpi<BM, BN>::kEarly || (p.diag & 256))) tile_epi_load<BM, BN, GNM>(p, m0, n0, true, pre);
  if (!kEpiEarly || (p.diag & 256)) tile_epi_load<BM, BN, GNM>(p, m0, n0, false, pre);   // the late placement
  __syncthreads();  // every wave is done reading the ring
  constexpr int LDE = WN + 8;
  bf16* es = reinterpret_cast<bf16*>(smem) + wid * WM * LDE;
  DC_LDS_ASSERT((wid * WM * LDE) * 2, WM * LDE * 2, (Cfg<BM, BN, 64, 2>::EPI));
  if constexpr (GNM == 3) {
    // LayerNorm folded in: y = rstd (acc - mean csum[c]) + cbias[c], the rows' (mean, rstd) from p.ln_stats, one
    // 16-row slice at a time (all MI slices' statistics at once cost the 128 x 128 tiles a wave per SIMD)
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float mu[4], rs[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long m = m0 + wm * WM + i * 16 + row_l + e;
        const bool in = m < M;
        mu[e] = in ? p.ln_stats[m * 2] : 0.0f;
        rs[e] = in ? p.ln_stats[m * 2 + 1] : 0.0f;
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float cs = pre.cv[j], cb = pre.cv2[j];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          es[(i * 16 + row_l + e) * LDE + j * 16 + col_l] = (bf16)(rs[e] * (acc[i][j][e] - mu[e] * cs) + cb);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float bv = pre.cv[j];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) es[(i * 16 + row_l + e) * LDE + j * 16 + col_l] = (bf16)(acc[i][j][e] + bv);
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  constexpr int GPR = WN / 8;
  if (p.geglu == 1) {
    // (h, gate) column pairs 8 + 8: raw pre-activation to y, h * gelu(gate) to y2 (torch's bf16 rounding:
    // gelu(gate) rounded, then the product)
    constexpr int PPR = WN / 16;
    for (int g = lane; g < WM * PPR; g += 64) {
      const int row = g / PPR, pc = g - (g / PPR) * PPR;
      const long m = m0 + wm * WM + row;
      const int c = n0 + wn * WN + pc * 16;
      if (m >= M || c >= p.cout) continue;
      float h[8], gt[8], o[8];
      load8(es + row * LDE + pc * 16, h);
      load8(es + row * LDE + pc * 16 + 8, gt);
      store8(p.y + m * p.ldy + c, h);
      store8(p.y + m * p.ldy + c + 8, gt);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = h[k] * (float)(bf16)gelu_f(gt[k]);
      store8(p.y2 + m * p.ldy2 + c / 2, o);
    }
    return;
  }
  if (p.geglu == 2 && p.geglu_n && n0 >= p.geglu_n) {
    // the residual half of the folded FF2 / proj_out input-gradient: plain columns into y2 (block-uniform: geglu_n is
    // a multiple of 256, every tile lies on one side)
    for (int g = lane; g < WM * GPR; g += 64) {
      const int row = g / GPR, cg = g - (g / GPR) * GPR;
      const long m = m0 + wm * WM + row;
      const int c = n0 + wn * WN + cg * 8;
      if (m >= M || c >= p.cout) continue;
      float v[8];
      load8(es + row * LDE + cg * 8, v);
      store8(p.y2 + m * p.ldy2 + (c - p.geglu_n), v);
    }
    return;
  }
  if (p.geglu == 2) {
    // dL/d(h * gelu(gate)) of 8 channels -> (dL/dh, dL/dgate) at their interleaved columns
#pragma unroll 2
    for (int g = lane; g < WM * GPR; g += 64) {
      const int row = g / GPR, cg = g - (g / GPR) * GPR;
      const long m = m0 + wm * WM + row;
      const int c = n0 + wn * WN + cg * 8;
      if (m >= M || c >= p.cout) continue;
      float d[8], h[8], gt[8], dh[8], dg[8];
      load8(es + row * LDE + cg * 8, d);
      const long col = (long)(c / 8) * 16;
      load8(p.aux + m * p.ldaux + col, h);
      load8(p.aux + m * p.ldaux + col + 8, gt);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        dh[k] = d[k] * (float)(bf16)gelu_f(gt[k]);
        const float dgel = (float)(bf16)(d[k] * h[k]);
        dg[k] = dgel * gelu_grad(gt[k]);
      }
      store8(p.y + m * p.ldy + col, dh);
      store8(p.y + m * p.ldy + col + 8, dg);
    }
    return;
  }
  if constexpr (GNM == 1 || GNM == 2) {
    // frames of the block's first and last row decide the block-uniform reduction form
    const long mA = m0 + wm * WM;
    const long mlast = min(M, m0 + BM) - 1;
    const GnTargetP& t0 = p.gn.t[0];
    const int fa = (int)fast_div((unsigned)m0, t0.hw_mul, t0.hw_shr);
    const int fb = (int)fast_div((unsigned)mlast, t0.hw_mul, t0.hw_shr);
    gn_epilogue_rows<GNM, WM, WN, BN, 2, LDSB>(p, smem, es, LDE, n0, wm, wn, lane, fa, fb, [&](int row) -> long {
      const long m = mA + row;
      return m < M ? m : -1;
    });
    return;
  }
  if (p.diag & 64) return;   // experiments only: no epilogue stores
  if constexpr (!TileEpi<BM, BN>::kRows || !kEpiEarly) {   // each row's operands loaded as it is stored
#pragma unroll 4
    for (int g = lane; g < WM * GPR; g += 64) {
      const int row = g / GPR, cg = g - (g / GPR) * GPR;
      const long m = m0 + wm * WM + row;
      const int c = n0 + wn * WN + cg * 8;
      if (m >= M || c >= p.cout) continue;
      float v[8];
      load8(es + row * LDE + cg * 8, v);
      epilogue_store(p, conv_pix(p, m), c, v, false);
    }
    return;
  }
  constexpr int RMAX = TileEpi<BM, BN>::RMAX;
  const int cg = lane % GPR, c = n0 + wn * WN + cg * 8;
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    if (pre.mrow[r] < 0) continue;
    const int row = (lane + 64 * r) / GPR;
    float v[8];
    load8(es + row * LDE + cg * 8, v);
    epilogue_store_pre(p, pre, r, c, v);
  }
}

// bijective XCD-aware remap of a linear block id: workgroups are dealt round-robin to the 8 XCDs by
// linear id, so XCD x = id % 8 gets the contiguous logical range x * total / 8 ...
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// SK: stream-K decomposition (its own instantiation: the segment loop's state would otherwise raise the
// register count -- and cut the occupancy -- of the plain / split-K kernel)
// GNM: the fused GroupNorm-statistics epilogue (p.gn; 1 forward, 2 backward), its own instantiations
// (conv_gemm_gn.hip) so that its registers do not lower the occupancy of the plain kernel (GNM 0)
template <int BM, int BN, int BK, int S, bool SMALLC, bool SK, int GNM>
__global__ __launch_bounds__(256) void conv_gemm_kernel(const ConvGemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[Cfg<BM, BN, BK, S>::LDS];
  f32x4 acc[BM / 32][BN / 32];
  typename TileEpi<BM, BN>::Pre pre;
  const int tiles_n = (p.cout + BN - 1) / BN;
  const int nk = p.ktot / BK;

  if constexpr (!SK) {
    // split-K (splits == 1: plain tiles).  Split-major logical order over the whole (tile, split)
    // grid: with K split 8 ways each XCD streams one K slice of A and W through its own L2 (each byte
    // fetched from HBM once); unsplit, each XCD gets a contiguous run of row tiles.
    const int tiles = gridDim.x, nblk = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int wk = xcd_remap(bid, nblk);
    const int tiles_m = tiles / tiles_n;
    int split, lb, tm, tn;
    if (p.nmajor) {
      // (column tile, split, row tile) with the row tile fastest: an XCD's contiguous range shares each (tn, split)
      // slice of W across all row tiles, so every weight byte leaves HBM for one XCD only
      tm = wk % tiles_m;
      const int rest = wk / tiles_m;
      split = rest % p.splits;
      tn = rest / p.splits;
      lb = tm * tiles_n + tn;
    } else {
      split = wk / tiles;
      lb = wk - split * tiles;
      tm = lb / tiles_n;
      tn = lb - tm * tiles_n;
    }
    const long m0 = (long)tm * BM;
    const int n0 = tn * BN;
    const int kc_begin = split * p.kps;
    const int kc_end = min(nk, kc_begin + p.kps);
    // the epilogue's column operands (and, where registers allow, its row operands) in flight under the main loop
    if (kEpiEarly && !(p.diag & 256)) {
      tile_epi_load<BM, BN, GNM>(p, m0, n0, false, pre);
      if (TileEpi<BM, BN>::kEarly) tile_epi_load<BM, BN, GNM>(p, m0, n0, true, pre);
    }
    tile_pass<BM, BN, BK, S, SMALLC>(p, smem, m0, n0, kc_begin, kc_end, acc);
    if (p.splits > 1 &&
        !tile_handoff<BM, BN>(p, smem, lb, split * tiles + lb, p.splits, [&](int sp) { return sp * tiles + lb; },
                              acc))
      return;
    tile_epilogue<BM, BN, GNM, Cfg<BM, BN, BK, S>::LDS>(p, smem, m0, n0, acc, pre);
  } else {
  // stream-K: the tiles x nk k-chunk iterations are dealt out as G equal contiguous ranges (logical
  // block b gets [b U / G, (b + 1) U / G)), so every block does the same MFMA work whatever the tile
  // count; a tile cut between blocks is finished by its last-arriving block (tile_handoff).  Slab
  // slots: 2b for block b's first segment, 2b + 1 for its last.
  const int G = gridDim.x;
  const long U = (long)p.splits * nk;  // p.splits carries the tile count in stream-K mode
  const int b = xcd_remap(blockIdx.x, G);
  long it = (long)b * U / G;
  const long start = it, end = (long)(b + 1) * U / G;
  // logical block holding iteration i: the largest b with b U / G <= i
  auto owner = [&](long i) { return (int)(((i + 1) * G - 1) / U); };
  while (it < end) {
    const int tile = (int)(it / nk);
    const int kb = (int)(it - (long)tile * nk);
    const int ke = (int)min((long)nk, kb + (end - it));
    int tm, tn;
    tile_coords(p, tile, p.splits / tiles_n, tiles_n, tm, tn);
    const long m0 = (long)tm * BM;
    const int n0 = tn * BN;
    if (kEpiEarly && !(p.diag & 256)) {
      tile_epi_load<BM, BN, GNM>(p, m0, n0, false, pre);
      if (TileEpi<BM, BN>::kEarly) tile_epi_load<BM, BN, GNM>(p, m0, n0, true, pre);
    }
    tile_pass<BM, BN, BK, S, SMALLC>(p, smem, m0, n0, kb, ke, acc);
    bool mine = true;
    if (kb != 0 || ke != nk) {
      const long t0 = (long)tile * nk;
      const int bf = owner(t0), bl = owner(t0 + nk - 1);
      const int slot = (it == start) ? 2 * b : 2 * b + 1;
      mine = tile_handoff<BM, BN>(
          p, smem, tile, slot, bl - bf + 1,
          [&](int i) { const int bb = bf + i; return ((long)bb * U / G >= t0) ? 2 * bb : 2 * bb + 1; }, acc);
    }
    if (mine) tile_epilogue<BM, BN, GNM, Cfg<BM, BN, BK, S>::LDS>(p, smem, m0, n0, acc, pre);
    it += ke - kb;
    __syncthreads();  // the ring / epilogue tile is free before the next segment's LDS-DMA
  }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Halo-tile direct 3x3 conv (stride 1, pad 1; mode 0 direct, mode 1 nearest upsample folded in; cin % 64 == 0).
//
// The im2col path above fills every 3x3 A row 9 times (once per tap) from L2; at batch 1 the UNet / TAESD convs
// are bound by that operand fill (32 FLOP per filled byte on a 64x64 tile).  Here a block owns a TH x TW
// spatial tile of output pixels (one frame) x BN output channels and walks the input channels in 64-wide
// chunks: per chunk it fills the (TH+2) x (TW+2) halo of the input ONCE into LDS and runs all 9 taps from it
// (the A fragment of tap (ky, kx) for output pixel (ty, tx) is halo row (ty+ky)(TW+2) + tx+kx: a per-lane LDS
// address), while the weights stream through an S-deep ring one (tap, chunk) slice of BN x 64 at a time.
// Per 64-channel chunk that is (TH+2)(TW+2) + 9 BN rows of 128 B for 2 TH TW BN 576 FLOP: 162 FLOP/B at
// 8x32 x 64 against 32 (64x64 im2col) and 64 (128x128 im2col).
//
// Pipeline: iteration i = (chunk c, tap t), i = 9 (c - c_begin) + t.  The halo of chunk c is issued with the
// weight slice of its tap 0, S - 1 iterations ahead like every weight slice (two halo slots: chunk c + 1's
// halo lands in the slot chunk c - 1 used, issued no earlier than (c, 1)).  Before iteration i the waves wait
// (counted vmcnt) until only the loads of iterations i+1 .. i+S-2 may be in flight: that retires iteration
// i's weights and its chunk's halo; one barrier per iteration.  Input channels split over blocks (split-K)
// are summed in split order by the last-arriving block (tile_handoff_g).  4 waves, WGM x WGN wave layout;
// BMP = TH TW padded to whole 16-row fragments per wave (pad rows compute garbage that is never stored).
template <int TH, int TW, int BN, int WGM, int WGN, int S>
struct HaloCfg {
  static_assert(WGM * WGN == 4, "4 waves");
  static constexpr int BM = TH * TW;
  static constexpr int BMP = ((BM + 16 * WGM - 1) / (16 * WGM)) * (16 * WGM);
  static constexpr int WM = BMP / WGM, WN = BN / WGN;
  static constexpr int MI = WM / 16, NJ = WN / 16;
  static_assert(WN % 16 == 0 && BN % 32 == 0, "BN");
  static constexpr int HW2 = TW + 2;
  static constexpr int HROWS = (TH + 2) * (TW + 2);
  static constexpr int LH = (HROWS + 31) / 32;   // block-wide 16-B LDS-DMA instructions per thread per halo
  static constexpr int LW = BN / 32;             // ... per weight slice
  static constexpr int RB = 128;                 // 64 bf16 channels per LDS row
  static constexpr int HALO = LH * 32 * RB;
  static constexpr int WST = BN * RB;
  // two halo slots: chunk c's halo is issued S - 1 iterations ahead of its tap 0, into the slot chunk c - 2
  // used, whose last read (its tap 8) precedes that issue for S <= 10
  static constexpr int RING = 2 * HALO + S * WST;
  static constexpr int EPI = 4 * WM * (WN + 8) * 2;
  static constexpr int LDS = RING > EPI ? RING : EPI;
  static_assert(S >= 2 && S <= 10, "ring depth (two halo slots)");
  static_assert((S - 2) * LW + LH <= 63, "vmcnt range");
};

// The main loop is unrolled over the 9 taps of a chunk, so every count below is a compile-time constant: at tap t
// of a chunk that is not the block's last, the loads younger than iteration i's are iterations i+1 .. i+S-2,
// (S-2) LW weight pieces plus one halo when t + S - 2 >= 9; in the last chunk only min(S-2, 8-t) iterations
// follow, none with a halo.  (A runtime-selected vmcnt was a ~450-cycle branch chain per iteration.)
template <int TH, int TW, int BN, int WGM, int WGN, int S, int SCHED, int GNM>
struct HaloBlock {
  using C = HaloCfg<TH, TW, BN, WGM, WGN, S>;
  static constexpr int MI = C::MI, NJ = C::NJ, WM = C::WM, WN = C::WN, RB = C::RB, LH = C::LH, LW = C::LW;
  static_assert(S <= 10, "two halo slots: the unrolled schedule assumes S - 1 <= 9");
  static constexpr int kOOB = (int)0x80000000u;

  const ConvGemmParams& p;
  char* smem;
  int lane, wid_s, wm, wn;
  int frame, oy0, ox0, n0, c_begin, c_end;
  int h_off[LH], h_off2[LH], b_off[LW], hbase[MI];
  __amdgpu_buffer_rsrc_t ra, ra2, rb;
  // issue cursor (scalar): the next iteration to load (its chunk, tap and weight slot)
  int q_c, q_t, q_slot;
  // compute cursor: the current chunk's halo slot and the current weight slot
  int cpar, wslot;
  f32x4 acc[MI][NJ];
  // epilogue operands loaded ahead (EpiPre): at kernel start where the row operands fit the registers
  static constexpr int GPR = WN / 8;
  static constexpr int RMAX = (WM * GPR + 63) / 64;
  static constexpr bool kEarly = RMAX <= 4;
  EpiPre<NJ, RMAX> pre;
  __device__ __forceinline__ long out_pix(int row) const {   // output pixel of wave row `row` (-1: outside)
    const int pl = wm * WM + row;
    const int ty = pl / TW, tx = pl - (pl / TW) * TW;
    const int oy = oy0 + ty, ox = ox0 + tx;
    if (pl >= C::BM || oy >= p.hout || ox >= p.wout) return -1;
    return ((long)frame * p.hout + oy) * p.wout + ox;
  }
  __device__ __forceinline__ void epi_load_rows() {
    if (GNM != 0) return;
    const int c = n0 + wn * WN + (lane % GPR) * 8;
    const bool full = c + 8 <= p.cout;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int g = lane + 64 * r;
      pre.mrow[r] = (g < WM * GPR && c < p.cout) ? out_pix(g / GPR) : -1;
      if (pre.mrow[r] >= 0 && full) {
        if (p.resid) pre.res[r] = *reinterpret_cast<const bf16x8*>(p.resid + pre.mrow[r] * p.ldr + c);
        if (p.mask) pre.msk[r] = *reinterpret_cast<const bf16x8*>(p.mask + pre.mrow[r] * p.ldmask + c);
      }
    }
    if (p.rowbias && full) pre.rb = *reinterpret_cast<const bf16x8*>(p.rowbias + (long)(*p.rowbias_idx) * p.rowbias_ld + c);
  }

  __device__ __forceinline__ void issue_halo(int c) {
    DC_LDS char* hb = (DC_LDS char*)smem + ((c - c_begin) & 1) * C::HALO;
    const int ch = c * 64;
    if (ch >= p.c1) {
#pragma unroll
      for (int j = 0; j < LH; ++j) buf_load_lds16(ra2, hb + (wid_s * 64 + 256 * j) * 16, h_off2[j], (ch - p.c1) * 2);
    } else {
#pragma unroll
      for (int j = 0; j < LH; ++j) buf_load_lds16(ra, hb + (wid_s * 64 + 256 * j) * 16, h_off[j], ch * 2);
    }
  }
  __device__ __forceinline__ void issue_w(int c, int t) {
    DC_LDS char* wb = (DC_LDS char*)smem + 2 * C::HALO + q_slot * C::WST;
    const int koff = (t * p.cin + c * 64) * 2;
#pragma unroll
    for (int j = 0; j < LW; ++j) buf_load_lds16(rb, wb + (wid_s * 64 + 256 * j) * 16, b_off[j], koff);
    q_slot = q_slot + 1 == S ? 0 : q_slot + 1;
  }
  // generic issue of the next iteration (prologue only)
  __device__ __forceinline__ void issue_next() {
    if (q_t == 0) issue_halo(q_c);
    issue_w(q_c, q_t);
    if (++q_t == 9) {
      q_t = 0;
      ++q_c;
    }
  }

  // one iteration (chunk c = current, tap T)
  template <int T, bool LAST>
  __device__ __forceinline__ void tap_step() {
    constexpr int K = LAST ? ((S - 2) < (8 - T) ? (S - 2) : (8 - T)) : (S - 2);
    constexpr int E = (!LAST && T + S - 2 >= 9) ? 1 : 0;
    vm_wait<K * LW + E * LH>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // load iteration i + S - 1: chunk + (T + S - 1 >= 9), tap (T + S - 1) % 9 (none past the block's last)
    constexpr int TT = T + S - 1;
    if constexpr (!LAST || TT < 9) {
      if constexpr (TT % 9 == 0) issue_halo(q_c);
      issue_w(q_c, TT % 9);
      if constexpr (TT % 9 == 8) ++q_c;
    }
    constexpr int KY = T / 3, KX = T % 3;
    constexpr int TOFF = KY * C::HW2 + KX;
    const char* ha = smem + cpar * C::HALO;
    const char* wbase = smem + 2 * C::HALO + wslot * C::WST;
    bf16x8 af[2][MI], bfr[2][NJ];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int ii = 0; ii < MI; ++ii) {
        const int r = hbase[ii] + TOFF;
        af[ks][ii] = *reinterpret_cast<const bf16x8*>(ha + r * RB + ((chunk ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj) {
        const int row = wn * WN + jj * 16 + (lane & 15);
        bfr[ks][jj] = *reinterpret_cast<const bf16x8*>(wbase + row * RB + ((chunk ^ (row & 7)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ii = 0; ii < MI; ++ii)
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj)
          acc[ii][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][ii], bfr[ks][jj], acc[ii][jj], 0, 0, 0);
    if constexpr (SCHED == 0) {
      // every fragment read of the tap ahead of its MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (MI + NJ), 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MI * NJ, 0);
    } else {
      // the first k-half's reads, then its MFMAs interleaved with the second k-half's reads, then the rest
      __builtin_amdgcn_sched_group_barrier(0x100, MI + NJ, 0);
#pragma unroll
      for (int q = 0; q < MI + NJ; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MI * NJ - (MI + NJ), 0);
    }
    wslot = wslot + 1 == S ? 0 : wslot + 1;
  }
  template <bool LAST, int... T>
  __device__ __forceinline__ void chunk_steps(std::integer_sequence<int, T...>) {
    (tap_step<T, LAST>(), ...);
  }

  __device__ __forceinline__ void run() {
    const int tid = threadIdx.x;
    lane = tid & 63;
    wid_s = __builtin_amdgcn_readfirstlane(tid >> 6);
    wm = (tid >> 6) / WGN;
    wn = (tid >> 6) % WGN;
    // ---- block -> (split, column tile, frame, tile row, tile column): split-major over the whole grid
    const int tiles_n = (p.cout + BN - 1) / BN;
    const int tiles_x = (p.wout + TW - 1) / TW, tiles_y = (p.hout + TH - 1) / TH;
    const int tiles = gridDim.x, nblk = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int wk = xcd_remap(bid, nblk);
    const int split = wk / tiles;
    const int lb = wk - split * tiles;
    const int sp_tile = lb / tiles_n, tn = lb - (lb / tiles_n) * tiles_n;
    frame = sp_tile / (tiles_y * tiles_x);
    const int trem = sp_tile - frame * (tiles_y * tiles_x);
    oy0 = (trem / tiles_x) * TH;
    ox0 = (trem - (trem / tiles_x) * tiles_x) * TW;
    n0 = tn * BN;
    const int nck = p.cin / 64;
    c_begin = split * p.kps;
    c_end = min(nck, c_begin + p.kps);
    const int nch = max(0, c_end - c_begin);

    // ---- per-lane LDS-DMA offsets: halo rows (fixed for the block; the chunk's channel offset rides in soffset)
    const int slot = tid & 7, r0 = tid >> 3;
#pragma unroll
    for (int j = 0; j < LH; ++j) {
      const int hr = r0 + 32 * j;
      const int hy = hr / C::HW2, hx = hr - (hr / C::HW2) * C::HW2;
      const int vy = oy0 - 1 + hy, vx = ox0 - 1 + hx;
      const bool ok = hr < C::HROWS && vy >= 0 && vy < p.hout && vx >= 0 && vx < p.wout;
      int iy = vy, ix = vx;
      if (p.mode == 1) {
        iy = ok ? (int)fast_div((unsigned)(vy * p.hin), p.h_mul, p.h_shr) : 0;
        ix = ok ? (int)fast_div((unsigned)(vx * p.win), p.w_mul, p.w_shr) : 0;
      }
      const int pix = (frame * p.hin + iy) * p.win + ix;
      const int sw = (slot ^ (hr & 7)) * 8;
      h_off[j] = ok ? (pix * p.ldx + sw) * 2 : kOOB;
      h_off2[j] = ok ? (pix * p.ldx2 + sw) * 2 : kOOB;
    }
#pragma unroll
    for (int j = 0; j < LW; ++j) {
      const int row = r0 + 32 * j;
      const int co = n0 + row;
      b_off[j] = co < p.cout ? (co * p.ktot + (slot ^ (row & 7)) * 8) * 2 : kOOB;
    }
    ra = buf_rsrc(p.x);
    ra2 = buf_rsrc(p.x2);
    rb = buf_rsrc(p.w);
    // per-lane halo row of each A fragment at tap (0, 0)
#pragma unroll
    for (int ii = 0; ii < MI; ++ii) {
      int pl = wm * WM + ii * 16 + (lane & 15);
      pl = pl < C::BM ? pl : 0;   // pad rows read a valid halo row; never stored
      const int ty = pl / TW, tx = pl - (pl / TW) * TW;
      hbase[ii] = ty * C::HW2 + tx;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the epilogue's column (and, where registers allow, row) operands in flight under the main loop
    if (kEpiEarly && !(p.diag & 256)) {
      epi_cols<0>(p, n0 + wn * WN + (lane & 15), pre);
      if (kEarly) epi_load_rows();
    }

    q_c = c_begin;
    q_t = 0;
    q_slot = 0;
    const int NI = nch * 9;
    for (int s = 0; s < S - 1 && s < NI; ++s) issue_next();
    // after the prologue the issue cursor sits at iteration S - 1: chunk c_begin + (S-1)/9 ... (S - 1 <= 9)
    cpar = 0;
    wslot = 0;
    for (int c = 0; c < nch; ++c) {
      // keep the 9 taps' fragment addresses out of registers across chunks (hoisted, they cost 9 x 2 x MI VGPRs
      // and spilled the 9-fragment variants): recomputed per tap, in the MFMAs' VALU shadow
#pragma unroll
      for (int ii = 0; ii < MI; ++ii) asm volatile("" : "+v"(hbase[ii]));
      if (c + 1 < nch) chunk_steps<false>(std::make_integer_sequence<int, 9>{});
      else chunk_steps<true>(std::make_integer_sequence<int, 9>{});
      cpar ^= 1;
    }
    vm_wait<0>();

    if (p.splits > 1 && !tile_handoff_g<MI, NJ>(p, smem, lb, split * tiles + lb, p.splits,
                                                [&](int sp) { return sp * tiles + lb; }, acc))
      return;
    epilogue();
  }

  // ---- epilogue: bias in fp32, bf16 per-wave LDS tile, then 16-B rows mapped to the tile's output pixels
  __device__ __forceinline__ void epilogue() {
    const int wid = threadIdx.x >> 6;
    const int col_l = lane & 15, row_l = (lane >> 4) * 4;
    if (kEpiEarly && (!kEarly || (p.diag & 256))) epi_load_rows();
    if (!kEpiEarly || (p.diag & 256)) epi_cols<0>(p, n0 + wn * WN + (lane & 15), pre);   // the late placement
    __syncthreads();
    constexpr int LDE = WN + 8;
    bf16* es = reinterpret_cast<bf16*>(smem) + wid * WM * LDE;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float bv = pre.cv[j];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) es[(i * 16 + row_l + q) * LDE + j * 16 + col_l] = (bf16)(acc[i][j][q] + bv);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    constexpr int GPR = WN / 8;
    if constexpr (GNM != 0) {
      // the tile lies in one frame
      const long pix0 = ((long)frame * p.hout + oy0) * p.wout + ox0;
      const GnTargetP& t0 = p.gn.t[0];
      const int fr = (int)fast_div((unsigned)pix0, t0.hw_mul, t0.hw_shr);
      gn_epilogue_rows<GNM, WM, WN, BN, WGM, C::LDS>(p, smem, es, LDE, n0, wm, wn, lane, fr, fr, [&](int row) -> long {
        const int pl = wm * WM + row;
        const int ty = pl / TW, tx = pl - (pl / TW) * TW;
        const int oy = oy0 + ty, ox = ox0 + tx;
        if (pl >= C::BM || oy >= p.hout || ox >= p.wout) return -1;
        return ((long)frame * p.hout + oy) * p.wout + ox;
      });
      return;
    }
    if (p.diag & 64) return;   // experiments only: no epilogue stores
    const int cg = lane % GPR, c = n0 + wn * WN + cg * 8;
    if constexpr (!kEpiEarly) {   // each row's operands loaded as it is stored
#pragma unroll 4
      for (int g = lane; g < WM * GPR; g += 64) {
        const long m = out_pix(g / GPR);
        if (m < 0 || c >= p.cout) continue;
        float v[8];
        load8(es + (g / GPR) * LDE + cg * 8, v);
        epilogue_store(p, m, c, v, false);
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      if (pre.mrow[r] < 0) continue;
      const int row = (lane + 64 * r) / GPR;
      float v[8];
      load8(es + row * LDE + cg * 8, v);
      epilogue_store_pre(p, pre, r, c, v);
    }
  }
};

template <int TH, int TW, int BN, int WGM, int WGN, int S, int SCHED, int GNM>
__global__ __launch_bounds__(256) void conv_halo_kernel(const ConvGemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[HaloCfg<TH, TW, BN, WGM, WGN, S>::LDS];
  HaloBlock<TH, TW, BN, WGM, WGN, S, SCHED, GNM> blk{p, smem};
  blk.run();
}

// halo variants: (TH, TW, BN, wave layout WGM x WGN, weight ring depth S)
struct HaloAlgo {
  int th, tw, bn, wgm, wgn, s, sched;
};
constexpr HaloAlgo kHaloAlgos[] = {
    // (sched 0: a tap's fragment reads all ahead of its MFMAs; 1: second k-half's reads under the first's MFMAs)
    {8, 32, 64, 4, 1, 8, 0},    // 256 px x 64: TAESD 64-channel levels, UNet level 0 (152 KB, 1 block / CU)
    {4, 32, 64, 2, 2, 6, 0},    // 128 px x 64 (104 KB)
    {4, 32, 32, 4, 1, 8, 0},    // 128 px x 32 (88 KB)
    {8, 16, 64, 4, 1, 6, 0},    // 128 px x 64, 16 wide (level 1: 48 columns) (96 KB)
    {6, 24, 64, 1, 4, 6, 0},    // 144 px x 64 (level 2: 18 x 24) (104 KB)
    {9, 12, 64, 1, 4, 8, 0},    // 108 px x 64 (level 3: the whole 9 x 12 frame) (104 KB)
    {9, 12, 32, 2, 2, 8, 0},    // 108 px x 32 (level 3) (72 KB, 2 blocks / CU)
    {8, 24, 32, 2, 2, 4, 0},    // 192 px x 32 (level 2) (88 KB)
    {8, 16, 64, 4, 1, 4, 0},    // 128 px x 64 (80 KB, 2 blocks / CU)
    {4, 32, 64, 2, 2, 3, 0},    // 128 px x 64 (80 KB, 2 blocks / CU)
    {8, 16, 64, 4, 1, 4, 1},    // the two-blocks-per-CU forms, interleaved schedule
    {4, 32, 64, 2, 2, 3, 1},
    {8, 32, 64, 4, 1, 8, 1},
    {6, 24, 64, 1, 4, 6, 1},
    // (round 4, external ids 62 ..) 192-px tiles at one block per CU with an 8-deep weight ring: at batch 1 the level-0
    // frame (72 x 96) is 36 such tiles, x 5 column tiles = 180 blocks, all resident at once (the 128-px tiles give 270
    // blocks, more than the CUs at one block each, so they run two blocks per CU on a 3-deep ring and the weight stream
    // keeps ~16 KB per CU in flight); 4 x 1 waves of 48 / 64 px x 64 channels
    {4, 48, 64, 4, 1, 8, 1},    // 6 x 50 halo (144 KB)
    {6, 32, 64, 4, 1, 8, 1},    // 8 x 34 halo (136 KB)
    {8, 24, 64, 4, 1, 8, 1},    // 10 x 26 halo (136 KB)
    {4, 48, 64, 4, 1, 8, 0},
    {6, 32, 64, 4, 1, 8, 0},
};

constexpr long kCounterBytes = 64 * 1024;
constexpr int kMaxSplitTiles = (int)(kCounterBytes / 4);

// algorithm table: tile (BM, BN), k-chunk BK and ring depth S
struct Algo {
  int bm, bn, bk, s;
};
constexpr Algo kAlgos[] = {{0, 0, 0, 0},       {128, 128, 64, 4}, {128, 64, 64, 5}, {64, 64, 64, 4},
                           {64, 128, 64, 4},   {128, 128, 64, 3}, {128, 128, 32, 3}, {128, 64, 32, 4},
                           {64, 64, 32, 4},    {256, 64, 32, 3},  {128, 128, 64, 2}, {128, 128, 32, 2},
                           {128, 64, 64, 2},   {64, 64, 64, 2},   {256, 128, 32, 2}, {128, 256, 32, 2},
                           {256, 64, 64, 2},   {128, 32, 64, 2},  {64, 32, 64, 2},
                           // deep rings (7 / 5 k-chunks in flight) for long-K shapes on small grids, where one
                           // block per CU is bound by the bytes it keeps in flight
                           {64, 64, 64, 8},    {128, 64, 64, 6},  {64, 128, 64, 6}, {64, 64, 32, 8},
                           // (round 3, algo ids 37 ..) rings that fill the LDS of two blocks per CU (S = 5 at
                           // 64x64: the round-2 abort did not reproduce, profiles/r03p), or of three at 64x64 S = 3
                           {64, 64, 64, 5},    {128, 64, 64, 3},  {64, 128, 64, 3}, {64, 32, 64, 6},
                           {128, 32, 64, 4},   {64, 64, 64, 3},
                           // (round 3, algo ids 59 ..) wide tiles: all 320 output channels of a short-K linear / conv
                           // in one block, so each A row is filled into LDS once instead of once per 64-wide column
                           // tile (the level-0 attention projections, M = 6912, K = N = 320)
                           {32, 320, 64, 2},   {64, 320, 64, 2},  {32, 320, 64, 3}};
// External algo ids (dc_conv_desc.algo; the tuned table stores them): 1 .. kNumBase the first kNumBase entries of
// kAlgos, kNumBase + 1 .. kNumBase + kNumHalo the halo variants, then the later kAlgos entries.
constexpr int kNumAlgos = 28;   // kAlgos entries behind external ids 1 .. kNumAll (the wide tiles come after)
constexpr int kNumBase = 22;
constexpr int kNumHalo = 14;   // halo variants behind external ids kNumBase + 1 .. kNumBase + kNumHalo
constexpr int kNumHaloX = sizeof(kHaloAlgos) / sizeof(kHaloAlgos[0]) - kNumHalo;   // ... and behind kHaloXFirst ..
constexpr int kNumAll = kNumAlgos + kNumHalo;
// the wide tiles (kAlgos[kNumAlgos + 1 ..]) take the external ids after the skinny (43 .. 54) and resident (55 .. 58)
// variants of conv_skinny.h (conv_gemm.hip checks the numbering)
constexpr int kWideFirst = 59;
constexpr int kNumWide = sizeof(kAlgos) / sizeof(kAlgos[0]) - 1 - kNumAlgos;
static_assert(kNumAll == 42, "external algo ids of the tuned tables");
constexpr int kHaloXFirst = kWideFirst + kNumWide;   // 62: the round-4 halo variants
__host__ __device__ constexpr bool algo_is_halo(int id) {
  return (id > kNumBase && id <= kNumBase + kNumHalo) || (id >= kHaloXFirst && id < kHaloXFirst + kNumHaloX);
}
// kHaloAlgos index of a halo external id
__host__ __device__ constexpr int halo_index(int id) { return id < kHaloXFirst ? id - kNumBase - 1 : kNumHalo + id - kHaloXFirst; }
// kAlgos index of an im2col external id
__host__ __device__ constexpr int algo_index(int id) {
  return id <= kNumBase ? id : (id <= kNumAll ? id - kNumHalo : id - kWideFirst + kNumAlgos + 1);
}
static_assert(kNumHalo + kNumHaloX == 19, "DC_HALO cases below");

template <int TH, int TW, int BN, int WGM, int WGN, int S, int SCHED, int GNM>
int launch_halo(ConvGemmParams& p, int splits, hipStream_t stream) {
  using Cf = HaloCfg<TH, TW, BN, WGM, WGN, S>;
  const long tiles_l = (long)p.nb * ((p.hout + TH - 1) / TH) * ((p.wout + TW - 1) / TW) * ((p.cout + BN - 1) / BN);
  if (tiles_l >= (1L << 30)) return DC_ERR_ARG;
  const int tiles = (int)tiles_l;
  const int nck = p.cin / 64;
  p.counters = reinterpret_cast<int*>(reinterpret_cast<char*>(p.ws) + (p.ws_bytes - kCounterBytes));
  splits = max(1, min(splits, nck));   // stream-K requests (< 0) run unsplit
  if (p.ws == nullptr || tiles > kMaxSplitTiles) splits = 1;
  while (splits > 1 && (long)splits * tiles * Cf::BMP * BN * 4 > p.ws_bytes - kCounterBytes) --splits;
  p.kps = (nck + splits - 1) / splits;
  splits = (nck + p.kps - 1) / p.kps;
  p.splits = splits;
  p.sk_blocks = 0;
  hipLaunchKernelGGL((conv_halo_kernel<TH, TW, BN, WGM, WGN, S, SCHED, GNM>), dim3(tiles, splits), dim3(256), 0, stream, p);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// the halo kernel's contract: 3x3, stride 1, pad 1, direct (input = output size) or nearest-upsample input,
// whole 64-channel chunks (both concat sources), no row list / GEGLU epilogue, 32-bit byte offsets
bool halo_eligible(const ConvGemmParams& p) {
  if (p.kh != 3 || p.kw != 3 || p.stride != 1 || p.pad != 1 || p.rows || p.geglu) return false;
  if (p.cin % 64 != 0 || p.ktot != 9 * p.cin) return false;
  if (p.c1 < p.cin && p.c1 % 64 != 0) return false;
  if (p.mode == 0 && (p.hin != p.hout || p.win != p.wout)) return false;
  if (p.mode != 0 && p.mode != 1) return false;
  const long ld = p.ldx > p.ldx2 ? p.ldx : p.ldx2;
  if ((long)p.nb * p.hin * p.win * ld * 2 >= (1L << 31)) return false;
  if ((long)p.cout * p.ktot * 2 >= (1L << 31)) return false;
  return true;
}

template <int BM, int BN, int BK, int S, int GNM>
int launch_algo(ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t stream) {
  const int tiles = (int)((M + BM - 1) / BM) * ((p.cout + BN - 1) / BN);
  const int nk = p.ktot / BK;
  p.counters = reinterpret_cast<int*>(reinterpret_cast<char*>(p.ws) + (p.ws_bytes - kCounterBytes));
  if (splits < 0) {
    // stream-K over -splits x 256 blocks (at most one per k-chunk iteration; two slab slots per block)
    long g = min((long)(-splits) * 256, (long)tiles * nk);
    while (g > 1 && 2 * g * BM * BN * 4 > p.ws_bytes - kCounterBytes) g -= 256 > g ? 1 : 256;
    if (p.ws != nullptr && tiles <= kMaxSplitTiles && g > 1) {
      p.sk_blocks = (int)g;
      p.splits = tiles;
      p.kps = nk;
      if (smallc)
        hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, S, true, true, GNM>), dim3((int)g), dim3(256), 0, stream, p);
      else
        hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, S, false, true, GNM>), dim3((int)g), dim3(256), 0, stream, p);
      DC_CHECK_LAUNCH();
      return DC_OK;
    }
    splits = 1;
  }
  p.sk_blocks = 0;
  splits = max(1, min(splits, nk));
  if (p.ws == nullptr || tiles > kMaxSplitTiles) splits = 1;
  while (splits > 1 && (long)splits * tiles * BM * BN * 4 > p.ws_bytes - kCounterBytes) --splits;
  p.kps = (nk + splits - 1) / splits;
  splits = (nk + p.kps - 1) / p.kps;
  p.splits = splits;
  if (smallc)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, S, true, false, GNM>), dim3(tiles, splits), dim3(256), 0, stream, p);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, S, false, false, GNM>), dim3(tiles, splits), dim3(256), 0, stream, p);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// heuristic when the caller does not choose: enough work units for the 256 CUs
void auto_algo(long M, int cout, int nk, int& algo, int& splits) {
  auto units = [&](int bm, int bn) { return (int)((M + bm - 1) / bm) * ((cout + bn - 1) / bn); };
  const bool narrow = (cout <= 64) || (((cout + 63) / 64) * 64 < ((cout + 127) / 128) * 128);
  if (cout <= 32) {
    algo = 17;  // 128x32: output-channel counts like TAESD's final conv (3)
  } else if (!narrow && units(128, 128) >= 192) {
    algo = 10;  // 128x128, BK 64, double-buffered (2 blocks / CU)
  } else if (units(128, 64) >= 160) {
    algo = 12;  // 128x64, BK 64, double-buffered
  } else {
    algo = 13;  // 64x64, BK 64, double-buffered
  }
  const Algo a = kAlgos[algo];
  const int u = units(a.bm, a.bn);
  splits = 1;
  if (u < 160 && nk >= 8) splits = min(min((320 + u - 1) / u, nk / 4), 32);
}


// variant dispatch (the plain instantiations in conv_gemm.hip, the GroupNorm-epilogue ones in conv_gemm_gn*.hip)
template <int GNM>
int launch_halo_idx(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  switch (i) {
#define DC_HALO(i)                                                                                              \
  case i:                                                                                                       \
    return launch_halo<kHaloAlgos[i].th, kHaloAlgos[i].tw, kHaloAlgos[i].bn, kHaloAlgos[i].wgm, kHaloAlgos[i].wgn, \
                       kHaloAlgos[i].s, kHaloAlgos[i].sched, GNM>(p, splits, s);
    DC_HALO(0) DC_HALO(1) DC_HALO(2) DC_HALO(3) DC_HALO(4) DC_HALO(5) DC_HALO(6) DC_HALO(7) DC_HALO(8)
    DC_HALO(9) DC_HALO(10) DC_HALO(11) DC_HALO(12) DC_HALO(13) DC_HALO(14) DC_HALO(15) DC_HALO(16) DC_HALO(17)
    DC_HALO(18)
#undef DC_HALO
    default: return DC_ERR_ARG;
  }
}
template <int GNM>
int launch_algo_idx(int algo, ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t s) {
  switch (algo) {
#define DC_ALGO(i) \
  case i: return launch_algo<kAlgos[i].bm, kAlgos[i].bn, kAlgos[i].bk, kAlgos[i].s, GNM>(p, M, splits, smallc, s);
    DC_ALGO(1) DC_ALGO(2) DC_ALGO(3) DC_ALGO(4) DC_ALGO(5) DC_ALGO(6) DC_ALGO(7) DC_ALGO(8) DC_ALGO(9) DC_ALGO(10)
    DC_ALGO(11) DC_ALGO(12) DC_ALGO(13) DC_ALGO(14) DC_ALGO(15) DC_ALGO(16) DC_ALGO(17) DC_ALGO(18) DC_ALGO(19)
    DC_ALGO(20) DC_ALGO(21) DC_ALGO(22) DC_ALGO(23) DC_ALGO(24) DC_ALGO(25) DC_ALGO(26) DC_ALGO(27) DC_ALGO(28)
#define DC_ALGO_WIDE(i)                                                                                        \
  case i:                                                                                                      \
    if constexpr (GNM == 0)                                                                                    \
      return launch_algo<kAlgos[i].bm, kAlgos[i].bn, kAlgos[i].bk, kAlgos[i].s, 0>(p, M, splits, smallc, s); \
    return DC_ERR_ARG;
    // the wide tiles have no fused-GroupNorm form (gn_epilogue_rows needs 64 % (WN / 8) == 0; WN = 160 here)
    DC_ALGO_WIDE(29) DC_ALGO_WIDE(30) DC_ALGO_WIDE(31)
#undef DC_ALGO_WIDE
#undef DC_ALGO
    default: return DC_ERR_ARG;
  }
}

}  // namespace

// the GroupNorm-epilogue instantiations (conv_gemm_gn.hip: mode 1, conv_gemm_gnb.hip: mode 2)
int conv_launch_halo_gn(int i, ConvGemmParams& p, int splits, hipStream_t s);
int conv_launch_algo_gn(int algo, ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t s);
int conv_launch_halo_gnb(int i, ConvGemmParams& p, int splits, hipStream_t s);
int conv_launch_algo_gnb(int algo, ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t s);
// the LayerNorm-folded instantiations (conv_gemm_ln.hip: im2col tiles)
int conv_launch_algo_ln(int algo, ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t s);

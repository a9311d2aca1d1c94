// GroupNorm(+SiLU) and LayerNorm forward / backward on NHWC rows (gfx950).
//
// GroupNorm (diffusers ResnetBlock2D norm1/norm2 + SiLU, Transformer2DModel.norm, conv_norm_out),
// two launches, all reductions in a fixed order (bitwise reproducible run to run):
//   stats     per (frame, pixel-chunk) block (<= 128 chunks per frame): 8 channels per thread in registers
//             over its rows, rows folded through LDS, channels folded into group partials -> [nb][nchunk][G][2]
//   apply     every block first folds its frame's chunk partials (fp64, fixed order) -> mean, rstd, then
//             normalises (+ SiLU), 16 B per lane.  (DC_GN_FUSED=0: a separate finalize launch, one block per
//             frame, does the fold instead.)
// Backward: the same with (sum gamma*dy', sum gamma*dy'*xhat) and dx = rstd*(g*dy' - a - xhat*b).
// Small group slices (UNet levels 2-3) take a single launch instead: one block per (frame, group),
// see gn_group_fwd_kernel.
// The input may be two sources (UNet skip concat): channels >= c1 come from x2.
#include "common.h"
#include "gn_acc.h"
#include "../../include/dcamd.h"

#include <initializer_list>
#include <stdlib.h>

namespace {

struct GNShape {
  const bf16* x;
  const bf16* x2;
  int ldx, ldx2, c1;
  int nb, hw, c, groups, cpg;
  int rows_per_chunk, nchunk;
  int pf;      // elementwise passes: first row's loads issued ahead of the in-block partial fold (DC_GN_PF=0: off)
  int apply_rows;  // rows per block of the elementwise passes
  int cgs, R;  // colgroups (c/8) and parallel rows per block of the elementwise passes
  int Rs;      // parallel rows per block of the statistics passes (cgs * Rs <= 1024 threads)
};

__device__ __forceinline__ void gn_load8(const GNShape& s, int n, int row, int c, float* f) {
  const long pix = (long)n * s.hw + row;
  const bf16* src = (c < s.c1) ? (s.x + pix * s.ldx + c) : (s.x2 + pix * s.ldx2 + (c - s.c1));
  load8(src, f);
}

// group of each of a thread's 8 channels c0 .. c0 + 7: one division per thread instead of eight (the
// elementwise passes are short enough that the per-thread setup shows in their time)
__device__ __forceinline__ void gn_groups8(int c0, int cpg, int (&g)[8]) {
  int q = c0 / cpg, r = c0 - q * cpg;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    g[k] = q;
    if (++r == cpg) {
      r = 0;
      ++q;
    }
  }
}

// fold per-thread channel partials (a, b)[8] across the R row-lanes, then into group partials
__device__ void gn_block_fold(const GNShape& s, const float* a, const float* b, float* sh, float* out) {
  // sh: [2][Rs][c] floats
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  const bool active = r0 < s.Rs;
  float* sa = sh;
  float* sb = sh + s.Rs * s.c;
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sa[r0 * s.c + cg * 8 + i] = a[i];
      sb[r0 * s.c + cg * 8 + i] = b[i];
    }
  }
  __syncthreads();
  // per channel: sum over row-lanes (fixed order) -> reuse row 0
  for (int ch = threadIdx.x; ch < s.c; ch += blockDim.x) {
    float ta = 0.0f, tb = 0.0f;
    for (int r = 0; r < s.Rs; ++r) { ta += sa[r * s.c + ch]; tb += sb[r * s.c + ch]; }
    sa[ch] = ta;
    sb[ch] = tb;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < s.groups; g += blockDim.x) {
    float ta = 0.0f, tb = 0.0f;
    for (int k = 0; k < s.cpg; ++k) { ta += sa[g * s.cpg + k]; tb += sb[g * s.cpg + k]; }
    out[g * 2] = ta;
    out[g * 2 + 1] = tb;
  }
}

// (sum, sumsq) -> (mean, rstd) [mode 0] or (sum a / cnt, sum b / cnt) [mode 1] of one group
__device__ __forceinline__ void gn_final_pair(double ta, double tb, double cnt, float eps, int mode, float* dst) {
  if (mode == 0) {
    const double mu = ta / cnt;
    double var = tb / cnt - mu * mu;
    if (var < 0.0) var = 0.0;
    dst[0] = (float)mu;
    dst[1] = (float)(1.0 / sqrt(var + (double)eps));
  } else {
    dst[0] = (float)(ta / cnt);
    dst[1] = (float)(tb / cnt);
  }
}

// Finalize at the head of the elementwise pass (no finalize launch): every block folds its frame's nchunk
// [G][2] chunk partials into grp[G][2] (LDS).  Thread t owns group pair t % GP (GP = G / 2, one 16-B
// vector per chunk) and sums chunks t / GP, t / GP + nthr / GP, ... in fp64 (8 vectors in flight); the
// nthr / GP column sums are then added in thread order.  The order is fixed, so every block -- and every
// run -- gets the same bits.  Needs G even and blockDim % GP == 0 (gn_fold_ok).  red: blockDim x 4 doubles.
__device__ void gn_fold_in_block(const GNShape& s, const float* part_n, int mode, float eps, double* red,
                                 float* grp) {
  const int GP = s.groups >> 1, nthr = blockDim.x, tid = threadIdx.x;
  const int gp = tid % GP, cstep = nthr / GP;
  double a0 = 0.0, b0 = 0.0, a1 = 0.0, b1 = 0.0;
  for (int c0 = tid / GP; c0 < s.nchunk; c0 += 8 * cstep) {
    f32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ch = c0 + j * cstep;
      v[j] = ch < s.nchunk ? *reinterpret_cast<const f32x4*>(part_n + (long)ch * s.groups * 2 + gp * 4)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a0 += v[j][0];
      b0 += v[j][1];
      a1 += v[j][2];
      b1 += v[j][3];
    }
  }
  red[tid * 4 + 0] = a0;
  red[tid * 4 + 1] = b0;
  red[tid * 4 + 2] = a1;
  red[tid * 4 + 3] = b1;
  __syncthreads();
  if (tid < s.groups) {
    const int pr = tid >> 1, h = (tid & 1) * 2;
    double ta = 0.0, tb = 0.0;
    for (int j = pr; j < nthr; j += GP) {
      ta += red[j * 4 + h];
      tb += red[j * 4 + h + 1];
    }
    gn_final_pair(ta, tb, (double)s.hw * s.cpg, eps, mode, grp + tid * 2);
  }
  __syncthreads();
}

// One-pass form (dc_groupnorm_*_acc): the frame's 2 G quantities accumulated by the producing convs' epilogues
// (gn_acc.h, exact sums over the replicas) -> grp[G][2] in LDS, as gn_fold_in_block leaves it.  red: 2 G doubles.
__device__ void gn_acc_groups(const GNShape& s, const unsigned long long* acc_n, int mode, float eps, double* red,
                              float* grp) {
  const int tid = threadIdx.x;
  const long rstride = (long)s.nb * s.groups * kGnPair;
  if (tid < 2 * s.groups) red[tid] = gn_acc_read(acc_n + (long)(tid >> 1) * kGnPair + (tid & 1) * kGnWords, rstride);
  __syncthreads();
  if (tid < s.groups) gn_final_pair(red[2 * tid], red[2 * tid + 1], (double)s.hw * s.cpg, eps, mode, grp + tid * 2);
  __syncthreads();
}

__global__ void gn_stats_kernel(GNShape s, float* part) {
  extern __shared__ float sh[];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < s.Rs) {
    const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
    // two rows' loads in flight per iteration; accumulation in row order
    for (int row = rbeg + r0; row < rend; row += 2 * s.Rs) {
      const bool two = row + s.Rs < rend;
      float f[8], f2[8];
      gn_load8(s, n, row, cg * 8, f);
      if (two) gn_load8(s, n, row + s.Rs, cg * 8, f2);
#pragma unroll
      for (int i = 0; i < 8; ++i) { a[i] += f[i]; b[i] += f[i] * f[i]; }
      if (two) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { a[i] += f2[i]; b[i] += f2[i] * f2[i]; }
      }
    }
  }
  gn_block_fold(s, a, b, sh, part + ((long)n * s.nchunk + chunk) * s.groups * 2);
}

// one block per frame, one wave per group (looping): fp64 fold of the chunk partials.
// mode 0: out = (mean, rstd) from (sum, sumsq); mode 1: out = (sum a / cnt, sum b / cnt)
__global__ void gn_finalize_kernel(GNShape s, const float* part, float eps, int mode, float* out) {
  // one wave per (frame, group): grid (ceil(groups / 4), nb) x 256 threads
  const int n = blockIdx.y, lane = threadIdx.x & 63;
  const double cnt = (double)s.hw * s.cpg;
  {
    const int g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (g >= s.groups) return;
    double ta = 0.0, tb = 0.0;
    // up to 8 chunk partials per lane in flight at once (a loop-carried chain of loads would pay one
    // memory round trip per 64 chunks); summation order per lane unchanged: k = lane, lane + 64, ...
    for (int k0 = lane; k0 < s.nchunk; k0 += 512) {
      float2 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = k0 + 64 * j;
        v[j] = k < s.nchunk ? *reinterpret_cast<const float2*>(part + (((long)n * s.nchunk + k) * s.groups + g) * 2)
                            : float2{0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ta += v[j].x;
        tb += v[j].y;
      }
    }
    for (int o = 32; o >= 1; o >>= 1) {
      ta += __shfl_xor(ta, o, 64);
      tb += __shfl_xor(tb, o, 64);
    }
    if (lane == 0) gn_final_pair(ta, tb, cnt, eps, mode, out + ((long)n * s.groups + g) * 2);
  }
}

// Elementwise passes: block (chunk, frame) with the stats kernel's thread layout -- each thread keeps
// one 8-channel group (cg = tid % cgs) over rows r0, r0 + R, ... -- so the per-channel coefficients
// are computed once per thread and the row loop carries no divisions.
// part != nullptr: the block first folds the frame's chunk partials itself (gn_fold_in_block) and block 0 of
// the frame stores (mean, rstd) to stats for the backward; otherwise stats comes from gn_finalize_kernel.
// acc != nullptr: the one-pass form, (mean, rstd) from the fused accumulators (gn_acc_groups)
__global__ void gn_apply_kernel(GNShape s, const float* part, float eps, float* stats, const float* gamma,
                                const float* beta, int silu, bf16* y, int ldy, const unsigned long long* acc) {
  extern __shared__ double gsh[];
  const int n = blockIdx.y;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  const float* st = stats + (long)n * s.groups * 2;
  const int rbeg = blockIdx.x * s.apply_rows, rend = min(s.hw, rbeg + s.apply_rows), row0 = rbeg + r0;
  // the first row's loads go out with the fold's partial loads: one memory round trip before the first barrier
  const bool pf = s.pf && (part || acc) && r0 < s.R && row0 < rend;
  float f0[8];
  if (pf) gn_load8(s, n, row0, cg * 8, f0);
  if (acc) {
    float* grp = reinterpret_cast<float*>(gsh + 2 * s.groups);
    gn_acc_groups(s, acc + (long)n * s.groups * kGnPair, 0, eps, gsh, grp);
    if (blockIdx.x == 0 && threadIdx.x < s.groups * 2) stats[(long)n * s.groups * 2 + threadIdx.x] = grp[threadIdx.x];
    st = grp;
  } else if (part) {
    float* grp = reinterpret_cast<float*>(gsh + blockDim.x * 4);
    gn_fold_in_block(s, part + (long)n * s.nchunk * s.groups * 2, 0, eps, gsh, grp);
    if (blockIdx.x == 0 && threadIdx.x < s.groups * 2) stats[(long)n * s.groups * 2 + threadIdx.x] = grp[threadIdx.x];
    st = grp;
  }
  if (r0 >= s.R) return;
  float mu[8], rs[8], ga[8], be[8];
  int gk[8];
  gn_groups8(cg * 8, s.cpg, gk);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k, g = gk[k];
    mu[k] = st[g * 2];
    rs[k] = st[g * 2 + 1];
    ga[k] = gamma[c];
    be[k] = beta[c];
  }
  for (int row = row0; row < rend; row += s.R) {
    float f[8];
    if (pf && row == row0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = f0[k];
    } else {
      gn_load8(s, n, row, cg * 8, f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = (f[k] - mu[k]) * rs[k] * ga[k] + be[k];
      if (silu) v = silu_f((float)(bf16)v);
      f[k] = v;
    }
    store8(y + ((long)n * s.hw + row) * ldy + cg * 8, f);
  }
}

// backward statistics: (sum g dy', sum g dy' xhat) per group, dy' = dy * silu'(y) with y = gn(x) rounded
// to bf16 and dy' rounded to bf16, as autograd does on bf16
__global__ void gn_bwd_stats_kernel(GNShape s, const float* stats, const float* gamma, const float* beta, int silu,
                                    const bf16* dy, int lddy, float* part) {
  extern __shared__ float sh[];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < s.Rs) {
    // per-thread channel coefficients, once (the row loop carries no divisions or table loads)
    float mu[8], rsd[8], ga[8], be[8];
    int gk[8];
    gn_groups8(cg * 8, s.cpg, gk);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = cg * 8 + i, g = gk[i];
      mu[i] = stats[((long)n * s.groups + g) * 2];
      rsd[i] = stats[((long)n * s.groups + g) * 2 + 1];
      ga[i] = gamma[c];
      be[i] = beta[c];
    }
    const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
    for (int row = rbeg + r0; row < rend; row += s.Rs) {
      float f[8], d[8];
      gn_load8(s, n, row, cg * 8, f);
      load8(dy + ((long)n * s.hw + row) * lddy + cg * 8, d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xhat = (f[i] - mu[i]) * rsd[i];
        float dd = d[i];
        if (silu) {
          const float yv = (float)(bf16)(xhat * ga[i] + be[i]);
          dd = (float)(bf16)(dd * silu_grad(yv));
        }
        const float gd = dd * ga[i];
        a[i] += gd;
        b[i] += gd * xhat;
      }
    }
  }
  gn_block_fold(s, a, b, sh, part + ((long)n * s.nchunk + chunk) * s.groups * 2);
}

// part != nullptr: (ma, mb) folded by the block itself from the frame's chunk partials (gn_fold_in_block),
// otherwise read from ab (gn_finalize_kernel)
// acc != nullptr: the one-pass form (dy = the producer's stored dy', silu 0), (ma, mb) from the fused accumulators
__global__ void gn_bwd_apply_kernel(GNShape s, const float* stats, const float* gamma, const float* beta, int silu,
                                    const bf16* dy, int lddy, const float* part, const float* ab, bf16* dx, int lddx,
                                    const bf16* add1, int ldadd1, const bf16* add2, int ldadd2,
                                    const unsigned long long* acc) {
  extern __shared__ double gsh[];
  const int n = blockIdx.y;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  const float* abn = ab + (long)n * s.groups * 2;
  const int rbeg = blockIdx.x * s.apply_rows, rend = min(s.hw, rbeg + s.apply_rows), row0 = rbeg + r0;
  const bool pf = s.pf && (part || acc) && r0 < s.R && row0 < rend;  // as gn_apply_kernel
  float f0[8], d0[8], e10[8], e20[8];   // (the first row's residual inputs too: no second round trip after the fold)
  if (pf) {
    gn_load8(s, n, row0, cg * 8, f0);
    load8(dy + ((long)n * s.hw + row0) * lddy + cg * 8, d0);
    if (add1) load8(add1 + ((long)n * s.hw + row0) * ldadd1 + cg * 8, e10);
    if (add2) load8(add2 + ((long)n * s.hw + row0) * ldadd2 + cg * 8, e20);
  }
  if (acc) {
    float* grp = reinterpret_cast<float*>(gsh + 2 * s.groups);
    gn_acc_groups(s, acc + (long)n * s.groups * kGnPair, 1, 0.0f, gsh, grp);
    abn = grp;
  } else if (part) {
    float* grp = reinterpret_cast<float*>(gsh + blockDim.x * 4);
    gn_fold_in_block(s, part + (long)n * s.nchunk * s.groups * 2, 1, 0.0f, gsh, grp);
    abn = grp;
  }
  if (r0 >= s.R) return;
  float mu[8], rs[8], ga[8], be[8], ma[8], mb[8];
  int gk[8];
  gn_groups8(cg * 8, s.cpg, gk);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k, g = gk[k];
    mu[k] = stats[((long)n * s.groups + g) * 2];
    rs[k] = stats[((long)n * s.groups + g) * 2 + 1];
    ma[k] = abn[g * 2];
    mb[k] = abn[g * 2 + 1];
    ga[k] = gamma[c];
    be[k] = beta[c];
  }
  for (int row = row0; row < rend; row += s.R) {
    const long pix = (long)n * s.hw + row;
    float f[8], d[8], out[8];
    if (pf && row == row0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        f[k] = f0[k];
        d[k] = d0[k];
      }
    } else {
      gn_load8(s, n, row, cg * 8, f);
      load8(dy + pix * lddy + cg * 8, d);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xhat = (f[k] - mu[k]) * rs[k];
      float dd = d[k];
      if (silu) {
        const float yv = (float)(bf16)(xhat * ga[k] + be[k]);
        dd = (float)(bf16)(dd * silu_grad(yv));
      }
      out[k] = rs[k] * (dd * ga[k] - ma[k] - xhat * mb[k]);
    }
    const bool first = pf && row == row0;
    if (add1) {
      float e[8];
      if (first) {
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = e10[k];
      } else {
        load8(add1 + pix * ldadd1 + cg * 8, e);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) out[k] = (float)(bf16)out[k] + e[k];
    }
    if (add2) {
      float e[8];
      if (first) {
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = e20[k];
      } else {
        load8(add2 + pix * ldadd2 + cg * 8, e);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) out[k] = (float)(bf16)out[k] + e[k];
    }
    store8(dx + pix * lddx + cg * 8, out);
  }
}

// ---- single-launch GroupNorm: one block per (frame, group), both passes inside the block.
// The 3-launch form pays two kernel boundaries and a cross-block fold per GN (≈ 10-15 µs per forward at
// every UNet level, whatever the size); a block that owns a whole group needs no hand-off at all.
// Thread (v, r0) reads VEC channels (the v-th vector of the group's cpg channels) of rows r0, r0 + RP,
// ..., U rows' loads in flight at once (one CU streams the whole group slice, so the pass is bound by
// the bytes it keeps in flight); sums go to fp64 through a fixed-order block reduction (bitwise
// reproducible).  Pass 1 stashes what it read in LDS (the slice is at most 138 KB per tensor at the
// C2 shapes; the host only takes this path when it fits), and pass 2 reads it back from there: each
// thread re-reads only its own slots, so no barrier guards the stash.  Blocks are dealt so that one XCD
// owns a contiguous range of groups (its L2 holds its own channel slice of each row).
template <int VEC>
using bfvec = __bf16 __attribute__((ext_vector_type(VEC)));
template <int VEC>
using fvec = float __attribute__((ext_vector_type(VEC)));

constexpr int kGroupThreads = 1024;
constexpr int kGroupRed = 32 * sizeof(double);          // reduction scratch in front of the stash
constexpr long kGroupLds = 160 * 1024;                   // LDS per workgroup on gfx950

__device__ __forceinline__ int gn_group_block(int nblk) {
  const int b = blockIdx.x;
  return (nblk & 7) ? b : (b & 7) * (nblk >> 3) + (b >> 3);
}

__device__ __forceinline__ const bf16* gn_group_src(const GNShape& s, int n, int ch, long& ld) {
  if (ch < s.c1) {
    ld = s.ldx;
    return s.x + (long)n * s.hw * s.ldx + ch;
  }
  ld = s.ldx2;
  return s.x2 + (long)n * s.hw * s.ldx2 + (ch - s.c1);
}

// fixed-order fp64 block reduction of (a, b) over the block's waves; result in every thread
__device__ __forceinline__ void gn_group_reduce(float a, float b, double* red, double& ta, double& tb) {
  double da = a, db = b;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    da += __shfl_xor(da, o, 64);
    db += __shfl_xor(db, o, 64);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w] = da;
    red[16 + w] = db;
  }
  __syncthreads();
  ta = 0.0;
  tb = 0.0;
  for (int k = 0; k < nw; ++k) {
    ta += red[k];
    tb += red[16 + k];
  }
}

template <int VEC, int U>
__global__ __launch_bounds__(kGroupThreads) void gn_group_fwd_kernel(GNShape s, int vpr, int RP, float eps,
                                                                    const float* gamma, const float* beta, int silu,
                                                                    bf16* y, int ldy, float* stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* red = reinterpret_cast<double*>(smem);
  bfvec<VEC>* stash = reinterpret_cast<bfvec<VEC>*>(smem + kGroupRed);
  const int L = gn_group_block(s.nb * s.groups);
  const int n = L / s.groups, g = L % s.groups;
  const int v = threadIdx.x % vpr, r0 = threadIdx.x / vpr;
  const bool act = r0 < RP;
  const int ch = g * s.cpg + v * VEC;
  long ld;
  const bf16* src = gn_group_src(s, n, ch, ld);
  // the per-channel vectors go out with pass 1's loads (read after the block reduction they were one more round trip,
  // profiles/r06w: -12 us per step over the 41 forward group launches)
  float ga[VEC], be[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    ga[i] = gamma[ch + i];
    be[i] = beta[ch + i];
  }
  float s1 = 0.0f, s2 = 0.0f;
  if (act) {
    for (int r = r0; r < s.hw; r += RP * U) {
      bfvec<VEC> raw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r + u * RP;
        raw[u] = row < s.hw ? *reinterpret_cast<const bfvec<VEC>*>(src + row * ld) : bfvec<VEC>{};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r + u * RP;
        if (row < s.hw) stash[row * vpr + v] = raw[u];
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float f = (float)raw[u][i];
          s1 += f;
          s2 += f * f;
        }
      }
    }
  }
  double ta, tb;
  gn_group_reduce(s1, s2, red, ta, tb);
  const double cnt = (double)s.hw * s.cpg;
  const double mu_d = ta / cnt;
  double var = tb / cnt - mu_d * mu_d;
  if (var < 0.0) var = 0.0;
  const float mu = (float)mu_d, rs = (float)(1.0 / sqrt(var + (double)eps));
  if (threadIdx.x == 0) {
    stats[((long)n * s.groups + g) * 2] = mu;
    stats[((long)n * s.groups + g) * 2 + 1] = rs;
  }
  if (!act) return;
  bf16* dst = y + (long)n * s.hw * ldy + ch;
  for (int row = r0; row < s.hw; row += RP) {
    const bfvec<VEC> raw = stash[row * vpr + v];
    bfvec<VEC> o;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float t = ((float)raw[i] - mu) * rs * ga[i] + be[i];
      if (silu) t = silu_f((float)(bf16)t);
      o[i] = (bf16)t;
    }
    *reinterpret_cast<bfvec<VEC>*>(dst + (long)row * ldy) = o;
  }
}

template <int VEC, int U>
__global__ __launch_bounds__(kGroupThreads) void gn_group_bwd_kernel(GNShape s, int vpr, int RP, const float* stats,
                                                                    const float* gamma, const float* beta, int silu,
                                                                    const bf16* dy, int lddy, bf16* dx, int lddx,
                                                                    const bf16* add1, int ldadd1, const bf16* add2,
                                                                    int ldadd2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* red = reinterpret_cast<double*>(smem);
  bfvec<VEC>* sx = reinterpret_cast<bfvec<VEC>*>(smem + kGroupRed);
  // pass 1 keeps g dy' (fp32) next to x, so pass 2 does not recompute the SiLU gradient (an exact-division sigmoid
  // per element, the kernel's VALU bulk on the one CU that owns the group)
  fvec<VEC>* sg = reinterpret_cast<fvec<VEC>*>(
      smem + ((kGroupRed + (long)s.hw * vpr * VEC * 2 + 31) & ~31L));   // (32-B aligned: the host adds 32 bytes)
  const int L = gn_group_block(s.nb * s.groups);
  const int n = L / s.groups, g = L % s.groups;
  const int v = threadIdx.x % vpr, r0 = threadIdx.x / vpr;
  const bool act = r0 < RP;
  const int ch = g * s.cpg + v * VEC;
  long ld;
  const bf16* src = gn_group_src(s, n, ch, ld);
  const bf16* dsrc = dy + (long)n * s.hw * lddy + ch;
  const float mu = stats[((long)n * s.groups + g) * 2], rs = stats[((long)n * s.groups + g) * 2 + 1];
  float ga[VEC], be[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    ga[i] = act ? gamma[ch + i] : 0.0f;
    be[i] = act ? beta[ch + i] : 0.0f;
  }
  // dy' = dy * silu'(y) rounded as bf16 autograd does (as gn_bwd_stats_kernel); returns g * dy' and xhat
  auto elem = [&](float f, float d, int i, float& xh) {
    xh = (f - mu) * rs;
    float dd = d;
    if (silu) {
      const float yv = (float)(bf16)(xh * ga[i] + be[i]);
      dd = (float)(bf16)(dd * silu_grad(yv));
    }
    return dd * ga[i];
  };
  // the residual inputs of the thread's first kPA rows go out with the pass-1 loads (no second round trip after the
  // block reduction)
  constexpr int kPA = 4;
  bfvec<VEC> pa1[kPA], pa2[kPA];
  const long pix0 = (long)n * s.hw;
  if (act) {
#pragma unroll
    for (int j = 0; j < kPA; ++j) {
      const int row = r0 + j * RP;
      if (row < s.hw) {
        if (add1) pa1[j] = *reinterpret_cast<const bfvec<VEC>*>(add1 + (pix0 + row) * ldadd1 + ch);
        if (add2) pa2[j] = *reinterpret_cast<const bfvec<VEC>*>(add2 + (pix0 + row) * ldadd2 + ch);
      }
    }
  }
  float sa = 0.0f, sb = 0.0f;
  if (act) {
    for (int r = r0; r < s.hw; r += RP * U) {
      bfvec<VEC> rx[U], rd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r + u * RP;
        const bool ok = row < s.hw;
        rx[u] = ok ? *reinterpret_cast<const bfvec<VEC>*>(src + row * ld) : bfvec<VEC>{};
        rd[u] = ok ? *reinterpret_cast<const bfvec<VEC>*>(dsrc + (long)row * lddy) : bfvec<VEC>{};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r + u * RP;
        if (row >= s.hw) continue;
        sx[row * vpr + v] = rx[u];
        fvec<VEC> gv;
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          float xh;
          const float gd = elem((float)rx[u][i], (float)rd[u][i], i, xh);
          gv[i] = gd;
          sa += gd;
          sb += gd * xh;
        }
        sg[row * vpr + v] = gv;
      }
    }
  }
  double ta, tb;
  gn_group_reduce(sa, sb, red, ta, tb);
  const double cnt = (double)s.hw * s.cpg;
  const float ma = (float)(ta / cnt), mb = (float)(tb / cnt);
  if (!act) return;
  bf16* dst = dx + (long)n * s.hw * lddx + ch;
  for (int row = r0, j = 0; row < s.hw; row += RP, ++j) {
    const bfvec<VEC> rx = sx[row * vpr + v];
    const fvec<VEC> gv = sg[row * vpr + v];
    float out[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float xh = ((float)rx[i] - mu) * rs;   // as elem() forms it
      out[i] = rs * (gv[i] - ma - xh * mb);
    }
    if (add1) {
      bfvec<VEC> e;
      if (j < kPA) {
#pragma unroll
        for (int q = 0; q < kPA; ++q)
          if (q == j) e = pa1[q];   // (static register indexing)
      } else {
        e = *reinterpret_cast<const bfvec<VEC>*>(add1 + (pix0 + row) * ldadd1 + ch);
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) out[i] = (float)(bf16)out[i] + (float)e[i];
    }
    if (add2) {
      bfvec<VEC> e;
      if (j < kPA) {
#pragma unroll
        for (int q = 0; q < kPA; ++q)
          if (q == j) e = pa2[q];
      } else {
        e = *reinterpret_cast<const bfvec<VEC>*>(add2 + (pix0 + row) * ldadd2 + ch);
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) out[i] = (float)(bf16)out[i] + (float)e[i];
    }
    bfvec<VEC> o;
#pragma unroll
    for (int i = 0; i < VEC; ++i) o[i] = (bf16)out[i];
    *reinterpret_cast<bfvec<VEC>*>(dst + (long)row * lddx) = o;
  }
}

bool gn_make_shape(GNShape& s, const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c,
                   int groups) {
  if (!x || nb <= 0 || hw <= 0 || c <= 0 || groups <= 0 || groups > 64) return false;
  if (c % groups != 0 || c % 8 != 0 || c > 8 * 1024) return false;
  if (ldx % 8 || (x2 && (ldx2 % 8 || c1 % 8))) return false;
  s.x = (const bf16*)x;
  s.x2 = (const bf16*)(x2 ? x2 : x);
  s.ldx = ldx;
  s.ldx2 = x2 ? ldx2 : ldx;
  s.c1 = x2 ? c1 : (1 << 30);
  s.nb = nb;
  s.hw = hw;
  s.c = c;
  s.groups = groups;
  s.cpg = c / groups;
  s.cgs = c / 8;
  s.R = max(1, 256 / s.cgs);
  // statistics: up to 1024-thread blocks (the block fold's LDS, 2 Rs c floats, stays <= 64 KB), at most 128
  // chunks per frame so that the elementwise pass can fold a frame's partials itself (gn_fold_in_block)
  s.Rs = max(1, 1024 / s.cgs);
  const int target_blocks = max(8, min(128, 512 / nb));
  s.rows_per_chunk = max(s.Rs, (hw + target_blocks - 1) / target_blocks);
  s.rows_per_chunk = ((s.rows_per_chunk + s.Rs - 1) / s.Rs) * s.Rs;
  s.nchunk = (hw + s.rows_per_chunk - 1) / s.rows_per_chunk;
  // elementwise passes: ~1024 blocks over the launch, at least R and at most 64 rows per block
  const int bpf = max(1, 1024 / nb);
  s.apply_rows = min(64, max(s.R, (hw + bpf - 1) / bpf));
  s.apply_rows = ((s.apply_rows + s.R - 1) / s.R) * s.R;
  {
    const char* e = getenv("DC_GN_PF");  // host side, read per call (graphs capture the choice)
    s.pf = (e && atoi(e) == 0) ? 0 : 1;
  }
  return true;
}

// workspace layout: [partials nb*nchunk*G*2][ab nb*G*2]
inline long gn_part_floats(const GNShape& s) { return (long)s.nb * s.nchunk * s.groups * 2; }

// The elementwise pass folds the partials itself (two launches) when G is even and its block is a multiple
// of G / 2 threads; DC_GN_FUSED=0 keeps the separate finalize launch (A/B and tests).  Returns the dynamic
// LDS of the elementwise pass (0: separate finalize).
size_t gn_fold_lds(const GNShape& s) {
  if (const char* env = getenv("DC_GN_FUSED"))
    if (atoi(env) == 0) return 0;
  const int threads = s.cgs * s.R;
  if (s.groups % 2 || threads % (s.groups / 2)) return 0;
  return (size_t)threads * 4 * sizeof(double) + (size_t)s.groups * 2 * sizeof(float);
}

// Single-launch path selection: widest vector (8 / 4 / 2 channels) that divides the group and keeps
// every operand aligned; 0 = take the 3-launch form.  Taken when the group slice of each stashed tensor
// (hw * cpg * 2 bytes; the forward stashes x, the backward x and dy) is at most `cap` bytes: one CU
// streams the slice with `cpg`-wide row segments (a fraction of each 128-B line), so the single launch
// only wins where the slice is small -- measured (tools/gn_bench.py) up to ~70 KB forward, ~35 KB
// backward at the UNet shapes.  DC_GN_GROUP=0 forces the 3-launch form, DC_GN_GROUP=<bytes> sets the
// cap, DC_GN_GROUP=-1 lifts it to the LDS limit (A/B and tests).
int gn_group_vec(const GNShape& s, int tensors, long cap, std::initializer_list<const void*> ptrs) {
  if (const char* env = getenv("DC_GN_GROUP")) {   // read per call (host side only; graphs capture the choice)
    const long v = atol(env);
    if (v == 0) return 0;
    cap = v < 0 ? kGroupLds : v;
  }
  const long slice = (long)s.hw * s.cpg * 2;
  if (slice > cap || tensors * slice + kGroupRed + 32 > kGroupLds) return 0;
  for (int vec = 8; vec >= 2; vec >>= 1) {
    if (s.cpg % vec || s.cpg / vec > kGroupThreads) continue;
    bool ok = true;
    for (const void* p : ptrs) ok = ok && ((uintptr_t)p % (2 * vec) == 0);
    if (ok) return vec;
  }
  return 0;
}
constexpr long kGroupCapFwd = 72 * 1024, kGroupCapBwd = 36 * 1024;

// the stash may exceed the default 64 KB dynamic-LDS limit: raise it once per instantiation
#define DC_GN_GROUP_LAUNCH(KERNEL, ...)                                                                      \
  do {                                                                                                        \
    static const hipError_t attr_ = hipFuncSetAttribute(reinterpret_cast<const void*>(&KERNEL),              \
                                                        hipFuncAttributeMaxDynamicSharedMemorySize,           \
                                                        (int)(kGroupLds - kGroupRed));                        \
    (void)attr_;                                                                                              \
    hipLaunchKernelGGL(KERNEL, grid, blk, lds, st, __VA_ARGS__);                                              \
  } while (0)

}  // namespace

extern "C" long long dc_groupnorm_ws_bytes(int nb, int hw, int c, int groups) {
  GNShape s;
  static const bf16 dummy[8] = {};
  if (!gn_make_shape(s, dummy, c, nullptr, 0, 0, nb, hw, c, groups)) return -1;
  return (gn_part_floats(s) + (long)nb * groups * 2) * (long long)sizeof(float);
}

extern "C" int dc_groupnorm_fwd(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c,
                                int groups, float eps, const float* gamma, const float* beta, int silu, void* y,
                                int ldy, float* stats, float* ws, void* stream) {
  GNShape s;
  if (!gn_make_shape(s, x, ldx, x2, ldx2, c1, nb, hw, c, groups) || !y || !gamma || !beta || !ws || !stats)
    return DC_ERR_ARG;
  if (ldy % 8) return DC_ERR_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  if (const int vec = gn_group_vec(s, 1, kGroupCapFwd, {s.x, s.x2, y})) {
    const int vpr = s.cpg / vec, RP = kGroupThreads / vpr;
    const dim3 grid(nb * groups), blk(kGroupThreads);
    const size_t lds = kGroupRed + (size_t)hw * s.cpg * 2;
    // U: 128 B of loads in flight per thread
    if (vec == 8)
      DC_GN_GROUP_LAUNCH((gn_group_fwd_kernel<8, 8>), s, vpr, RP, eps, gamma, beta, silu, (bf16*)y, ldy, stats);
    else if (vec == 4)
      DC_GN_GROUP_LAUNCH((gn_group_fwd_kernel<4, 16>), s, vpr, RP, eps, gamma, beta, silu, (bf16*)y, ldy, stats);
    else
      DC_GN_GROUP_LAUNCH((gn_group_fwd_kernel<2, 32>), s, vpr, RP, eps, gamma, beta, silu, (bf16*)y, ldy, stats);
    DC_CHECK_LAUNCH();
    return DC_OK;
  }
  const int threads = s.cgs * s.R, sthreads = s.cgs * s.Rs;
  const size_t lds = 2 * (size_t)s.Rs * s.c * sizeof(float);
  hipLaunchKernelGGL(gn_stats_kernel, dim3(s.nchunk, nb), dim3(sthreads), lds, st, s, ws);
  const size_t flds = gn_fold_lds(s);
  if (!flds)
    hipLaunchKernelGGL(gn_finalize_kernel, dim3((groups + 3) / 4, nb), dim3(256), 0, st, s, ws, eps, 0, stats);
  const dim3 agrid((hw + s.apply_rows - 1) / s.apply_rows, nb);
  hipLaunchKernelGGL(gn_apply_kernel, agrid, dim3(threads), flds, st, s, flds ? ws : nullptr, eps, stats, gamma,
                     beta, silu, (bf16*)y, ldy, (const unsigned long long*)nullptr);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_groupnorm_bwd(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c,
                                int groups, const float* gamma, const float* beta, int silu, const float* stats,
                                const void* dy, int lddy, void* dx, int lddx, const void* add1, int ldadd1,
                                const void* add2, int ldadd2, float* ws, void* stream) {
  GNShape s;
  if (!gn_make_shape(s, x, ldx, x2, ldx2, c1, nb, hw, c, groups) || !dy || !dx || !stats || !ws) return DC_ERR_ARG;
  if (lddy % 8 || lddx % 8 || (add1 && ldadd1 % 8) || (add2 && ldadd2 % 8)) return DC_ERR_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  // (the stash: x in bf16 and g dy' in fp32, three slices' worth)
  if (const int vec = gn_group_vec(s, 3, kGroupCapBwd, {s.x, s.x2, dy, dx, add1 ? add1 : dx, add2 ? add2 : dx})) {
    const int vpr = s.cpg / vec, RP = kGroupThreads / vpr;
    const dim3 grid(nb * groups), blk(kGroupThreads);
    const size_t lds = kGroupRed + 3 * (size_t)hw * s.cpg * 2 + 32;
#define DC_GN_GROUP_BWD(V, U)                                                                                   \
  DC_GN_GROUP_LAUNCH((gn_group_bwd_kernel<V, U>), s, vpr, RP, stats, gamma, beta, silu, (const bf16*)dy, lddy,  \
                     (bf16*)dx, lddx, (const bf16*)add1, ldadd1, (const bf16*)add2, ldadd2)
    if (vec == 8)
      DC_GN_GROUP_BWD(8, 4);
    else if (vec == 4)
      DC_GN_GROUP_BWD(4, 8);
    else
      DC_GN_GROUP_BWD(2, 16);
#undef DC_GN_GROUP_BWD
    DC_CHECK_LAUNCH();
    return DC_OK;
  }
  const int threads = s.cgs * s.R, sthreads = s.cgs * s.Rs;
  const size_t lds = 2 * (size_t)s.Rs * s.c * sizeof(float);
  float* ab = ws + gn_part_floats(s);
  hipLaunchKernelGGL(gn_bwd_stats_kernel, dim3(s.nchunk, nb), dim3(sthreads), lds, st, s, stats, gamma, beta, silu,
                     (const bf16*)dy, lddy, ws);
  const size_t flds = gn_fold_lds(s);
  if (!flds) hipLaunchKernelGGL(gn_finalize_kernel, dim3((groups + 3) / 4, nb), dim3(256), 0, st, s, ws, 0.0f, 1, ab);
  const dim3 agrid((hw + s.apply_rows - 1) / s.apply_rows, nb);
  hipLaunchKernelGGL(gn_bwd_apply_kernel, agrid, dim3(threads), flds, st, s, stats, gamma, beta, silu,
                     (const bf16*)dy, lddy, flds ? ws : nullptr, ab, (bf16*)dx, lddx, (const bf16*)add1, ldadd1,
                     (const bf16*)add2, ldadd2, (const unsigned long long*)nullptr);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// whether the fused statistics pay for this GroupNorm: not where the single-launch form (one block per (frame, group),
// the slice stashed in LDS) runs it -- its one launch costs about what the fused producer epilogue adds
// (tools/gn_fuse_bench.py)
extern "C" int dc_gn_fuse_pays(int hw, int c, int groups, int backward) {
  if (hw <= 0 || c <= 0 || groups <= 0 || c % groups) return 0;
  GNShape s;
  alignas(16) static const bf16 dummy[8] = {};
  if (!gn_make_shape(s, dummy, c, nullptr, 0, 0, 1, hw, c, groups)) return 0;
  return gn_group_vec(s, backward ? 3 : 1, backward ? kGroupCapBwd : kGroupCapFwd, {dummy}) ? 0 : 1;
}

extern "C" long long dc_gn_acc_bytes(int nb, int groups) {
  if (nb <= 0 || groups <= 0) return -1;
  return (long long)kGnReplicas * nb * groups * kGnPair * 8;
}

// one-pass GroupNorm from the fused statistics: the elementwise pass with the accumulator read at its head
extern "C" int dc_groupnorm_fwd_acc(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c,
                                    int groups, float eps, const float* gamma, const float* beta, int silu,
                                    const long long* acc, void* y, int ldy, float* stats, void* stream) {
  GNShape s;
  if (!gn_make_shape(s, x, ldx, x2, ldx2, c1, nb, hw, c, groups) || !y || !gamma || !beta || !acc || !stats)
    return DC_ERR_ARG;
  if (ldy % 8 || ((uintptr_t)acc & 7)) return DC_ERR_ALIGN;
  const int threads = s.cgs * s.R;
  if (threads < 2 * groups) return DC_ERR_ARG;
  const size_t lds = (size_t)groups * 2 * (sizeof(double) + sizeof(float));
  const dim3 agrid((hw + s.apply_rows - 1) / s.apply_rows, nb);
  hipLaunchKernelGGL(gn_apply_kernel, agrid, dim3(threads), lds, (hipStream_t)stream, s, (const float*)nullptr, eps,
                     stats, gamma, beta, silu, (bf16*)y, ldy, (const unsigned long long*)acc);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_groupnorm_bwd_acc(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c,
                                    int groups, const float* gamma, const float* stats, const long long* acc,
                                    const void* dyp, int lddy, void* dx, int lddx, const void* add1, int ldadd1,
                                    const void* add2, int ldadd2, void* stream) {
  GNShape s;
  if (!gn_make_shape(s, x, ldx, x2, ldx2, c1, nb, hw, c, groups) || !dyp || !dx || !stats || !gamma || !acc)
    return DC_ERR_ARG;
  if (lddy % 8 || lddx % 8 || (add1 && ldadd1 % 8) || (add2 && ldadd2 % 8) || ((uintptr_t)acc & 7))
    return DC_ERR_ALIGN;
  const int threads = s.cgs * s.R;
  if (threads < 2 * groups) return DC_ERR_ARG;
  const size_t lds = (size_t)groups * 2 * (sizeof(double) + sizeof(float));
  const dim3 agrid((hw + s.apply_rows - 1) / s.apply_rows, nb);
  hipLaunchKernelGGL(gn_bwd_apply_kernel, agrid, dim3(threads), lds, (hipStream_t)stream, s, stats, gamma, gamma, 0,
                     (const bf16*)dyp, lddy, (const float*)nullptr, stats, (bf16*)dx, lddx, (const bf16*)add1, ldadd1,
                     (const bf16*)add2, ldadd2, (const unsigned long long*)acc);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// ---------------------------------------------------------------- LayerNorm (one wave per row)
namespace {

// Every global load of a row is issued before the first use (clamped segment index: lanes past the row's end re-read
// its last segment and skip it at every use; the per-channel vectors as 16-B loads).  Guarded by the lane condition,
// the loads sat in divergent branches that the compiler closed with a wait each -- ~10-45 dependent round trips per
// row (profiles/r06s).
template <int MAXV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16* x, int ldx, long rows, int c, float eps, const float* gamma,
                              const float* beta, bf16* y, int ldy, float* stats) {
  const long row = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = c >> 3;
  bf16x8 xr[MAXV];
  f32x4 ga[MAXV][2], be[MAXV][2];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vc = min(lane + 64 * k, nv - 1);
    xr[k] = *reinterpret_cast<const bf16x8*>(x + row * ldx + vc * 8);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ga[k][h] = *reinterpret_cast<const f32x4*>(gamma + vc * 8 + 4 * h);
      be[k][h] = *reinterpret_cast<const f32x4*>(beta + vc * 8 + 4 * h);
    }
  }
  float v[MAXV][8];
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[k][i] = (float)xr[k][i];
        s += v[k][i];
      }
    }
  }
  const float mu = wave_sum(s) / c;
  float q = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = v[k][i] - mu; q += d * d; }
    }
  }
  const float rs = rsqrtf(wave_sum(q) / c + eps);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mu) * rs * ga[k][i >> 2][i & 3] + be[k][i >> 2][i & 3];
      store8(y + row * ldy + vi * 8, o);
    }
  }
  if (lane == 0 && stats) {
    stats[row * 2] = mu;
    stats[row * 2 + 1] = rs;
  }
}

template <int MAXV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16* x, int ldx, long rows, int c, const float* gamma, const float* stats,
                              const bf16* dy, int lddy, bf16* dx, int lddx, const bf16* add, int ldadd) {
  const long row = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = c >> 3;
  const float mu = stats[row * 2], rs = stats[row * 2 + 1];
  bf16x8 xr[MAXV], dr[MAXV], ar[MAXV];
  f32x4 ga[MAXV][2];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vc = min(lane + 64 * k, nv - 1);
    xr[k] = *reinterpret_cast<const bf16x8*>(x + row * ldx + vc * 8);
    dr[k] = *reinterpret_cast<const bf16x8*>(dy + row * lddy + vc * 8);
    if (add) ar[k] = *reinterpret_cast<const bf16x8*>(add + row * ldadd + vc * 8);
    if (gamma) {   // NULL: dy is gamma * dL/dy already
#pragma unroll
      for (int h = 0; h < 2; ++h) ga[k][h] = *reinterpret_cast<const f32x4*>(gamma + vc * 8 + 4 * h);
    }
  }
  float xh[MAXV][8], g[MAXV][8];
  float sa = 0.0f, sb = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[k][i] = ((float)xr[k][i] - mu) * rs;
        g[k][i] = gamma ? (float)dr[k][i] * ga[k][i >> 2][i & 3] : (float)dr[k][i];
        sa += g[k][i];
        sb += g[k][i] * xh[k][i];
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
      for (int i = 0; i < 8; ++i) o[i] = rs * (g[k][i] - ma - xh[k][i] * mb);
      if (add) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (float)(bf16)o[i] + (float)ar[k][i];
      }
      store8(dx + row * lddx + vi * 8, o);
    }
  }
}

}  // namespace

extern "C" int dc_layernorm_fwd(const void* x, int ldx, long long rows, int c, float eps, const float* gamma,
                                const float* beta, void* y, int ldy, float* stats, void* stream) {
  if (!x || !y || !gamma || !beta || rows <= 0 || c <= 0 || c % 8 || c > 2048 * 8) return DC_ERR_ARG;
  if (ldx % 8 || ldy % 8 || ((uintptr_t)gamma & 15) || ((uintptr_t)beta & 15)) return DC_ERR_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  const int wpb = 4;
  dim3 grid((unsigned)((rows + wpb - 1) / wpb));
  const int nv = c / 8;
  if (nv <= 64)
    hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, dim3(64 * wpb), 0, st, (const bf16*)x, ldx, (long)rows, c, eps, gamma,
                       beta, (bf16*)y, ldy, stats);
  else if (nv <= 192)
    hipLaunchKernelGGL(ln_fwd_kernel<3>, grid, dim3(64 * wpb), 0, st, (const bf16*)x, ldx, (long)rows, c, eps, gamma,
                       beta, (bf16*)y, ldy, stats);
  else if (nv <= 320)
    hipLaunchKernelGGL(ln_fwd_kernel<5>, grid, dim3(64 * wpb), 0, st, (const bf16*)x, ldx, (long)rows, c, eps, gamma,
                       beta, (bf16*)y, ldy, stats);
  else
    return DC_ERR_ARG;
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_layernorm_bwd(const void* x, int ldx, long long rows, int c, const float* gamma, const float* stats,
                                const void* dy, int lddy, void* dx, int lddx, const void* add, int ldadd,
                                void* stream) {
  if (!x || !dy || !dx || !stats || rows <= 0 || c <= 0 || c % 8) return DC_ERR_ARG;
  if (ldx % 8 || lddy % 8 || lddx % 8 || (add && ldadd % 8) || ((uintptr_t)gamma & 15)) return DC_ERR_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  const int wpb = 4;
  dim3 grid((unsigned)((rows + wpb - 1) / wpb));
  const int nv = c / 8;
  if (nv <= 64)
    hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, dim3(64 * wpb), 0, st, (const bf16*)x, ldx, (long)rows, c, gamma, stats,
                       (const bf16*)dy, lddy, (bf16*)dx, lddx, (const bf16*)add, ldadd);
  else if (nv <= 192)
    hipLaunchKernelGGL(ln_bwd_kernel<3>, grid, dim3(64 * wpb), 0, st, (const bf16*)x, ldx, (long)rows, c, gamma, stats,
                       (const bf16*)dy, lddy, (bf16*)dx, lddx, (const bf16*)add, ldadd);
  else if (nv <= 320)
    hipLaunchKernelGGL(ln_bwd_kernel<5>, grid, dim3(64 * wpb), 0, st, (const bf16*)x, ldx, (long)rows, c, gamma, stats,
                       (const bf16*)dy, lddy, (bf16*)dx, lddx, (const bf16*)add, ldadd);
  else
    return DC_ERR_ARG;
  DC_CHECK_LAUNCH();
  return DC_OK;
}

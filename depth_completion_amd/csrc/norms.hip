// GroupNorm(+SiLU) and LayerNorm forward / backward on NHWC rows (gfx950).
//
// GroupNorm (diffusers ResnetBlock2D norm1/norm2 + SiLU, Transformer2DModel.norm, conv_norm_out):
//   pass 1 (stats):  per (frame, pixel-chunk) block, channel sums in registers -> LDS -> group
//                    partial (sum, sumsq) slab  [nb][nchunk][G][2]
//   pass 2 (apply):  every block folds the slab for its frame (double) into (mean, rstd) per group,
//                    normalises its chunk, optional SiLU, writes bf16 (+ stats [nb][G][2] fp32).
// Backward follows the same two passes with (sum gamma*dy', sum gamma*dy'*xhat) partials.
// The input may be two sources (UNet skip concat): channels >= c1 come from x2.
#include "common.h"
#include "../../include/dcamd.h"

namespace {

struct GNShape {
  const bf16* x;
  const bf16* x2;
  int ldx, ldx2, c1;
  int nb, hw, c, groups, cpg;
  int rows_per_chunk, nchunk;
  int cgs, R;  // colgroups (c/8) and parallel rows per block
};

__device__ __forceinline__ void gn_load8(const GNShape& s, int n, int row, int c, float* f) {
  const long pix = (long)n * s.hw + row;
  const bf16* src = (c < s.c1) ? (s.x + pix * s.ldx + c) : (s.x2 + pix * s.ldx2 + (c - s.c1));
  load8(src, f);
}

__global__ void gn_stats_kernel(GNShape s, float* part) {
  extern __shared__ float sh[];  // [2*c]
  float* csum = sh;
  float* csq = sh + s.c;
  const int n = blockIdx.y, chunk = blockIdx.x;
  for (int i = threadIdx.x; i < 2 * s.c; i += blockDim.x) sh[i] = 0.0f;
  __syncthreads();
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  if (r0 < s.R) {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
    for (int row = rbeg + r0; row < rend; row += s.R) {
      float f[8];
      gn_load8(s, n, row, cg * 8, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) { a[i] += f[i]; b[i] += f[i] * f[i]; }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      atomicAdd(&csum[cg * 8 + i], a[i]);
      atomicAdd(&csq[cg * 8 + i], b[i]);
    }
  }
  __syncthreads();
  for (int g = threadIdx.x; g < s.groups; g += blockDim.x) {
    float ts = 0.0f, tq = 0.0f;
    for (int k = 0; k < s.cpg; ++k) { ts += csum[g * s.cpg + k]; tq += csq[g * s.cpg + k]; }
    float* dst = part + (((long)n * s.nchunk + chunk) * s.groups + g) * 2;
    dst[0] = ts;
    dst[1] = tq;
  }
}

// fold partial slabs of frame n into (mean, rstd) per group in LDS
__device__ void gn_fold_stats(const GNShape& s, const float* part, int n, float eps, float* mean, float* rstd) {
  for (int g = threadIdx.x; g < s.groups; g += blockDim.x) {
    double ts = 0.0, tq = 0.0;
    for (int k = 0; k < s.nchunk; ++k) {
      const float* src = part + (((long)n * s.nchunk + k) * s.groups + g) * 2;
      ts += src[0];
      tq += src[1];
    }
    const double cnt = (double)s.hw * s.cpg;
    const double mu = ts / cnt;
    double var = tq / cnt - mu * mu;
    if (var < 0.0) var = 0.0;
    mean[g] = (float)mu;
    rstd[g] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

__global__ void gn_apply_kernel(GNShape s, const float* part, float eps, const float* gamma, const float* beta,
                                int silu, bf16* y, int ldy, float* stats) {
  __shared__ float mean[64], rstd[64];
  const int n = blockIdx.y, chunk = blockIdx.x;
  gn_fold_stats(s, part, n, eps, mean, rstd);
  __syncthreads();
  if (chunk == 0 && stats) {
    for (int g = threadIdx.x; g < s.groups; g += blockDim.x) {
      stats[((long)n * s.groups + g) * 2] = mean[g];
      stats[((long)n * s.groups + g) * 2 + 1] = rstd[g];
    }
  }
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  if (r0 >= s.R) return;
  float gm[8], bt[8], mu[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = cg * 8 + i, g = c / s.cpg;
    gm[i] = gamma[c];
    bt[i] = beta[c];
    mu[i] = mean[g];
    rs[i] = rstd[g];
  }
  const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
  for (int row = rbeg + r0; row < rend; row += s.R) {
    float f[8];
    gn_load8(s, n, row, cg * 8, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = (f[i] - mu[i]) * rs[i] * gm[i] + bt[i];
      if (silu) v = silu_f((float)(bf16)v);
      f[i] = v;
    }
    store8(y + ((long)n * s.hw + row) * ldy + cg * 8, f);
  }
}

// dy' = dy * silu'(y) (y = gn(x) rounded to bf16, dy' rounded to bf16), as autograd does on bf16
__device__ __forceinline__ void gn_bwd_elem(const GNShape& s, int n, int row, int cg, const float* mu, const float* rs,
                                            const float* gm, const float* bt, int silu, const bf16* dy, int lddy,
                                            float* xh, float* gdy) {
  float f[8], d[8];
  gn_load8(s, n, row, cg * 8, f);
  load8(dy + ((long)n * s.hw + row) * lddy + cg * 8, d);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float xhat = (f[i] - mu[i]) * rs[i];
    float dd = d[i];
    if (silu) {
      const float yv = (float)(bf16)(xhat * gm[i] + bt[i]);
      dd = (float)(bf16)(dd * silu_grad(yv));
    }
    xh[i] = xhat;
    gdy[i] = dd * gm[i];
  }
}

__global__ void gn_bwd_stats_kernel(GNShape s, const float* stats, const float* gamma, const float* beta, int silu,
                                    const bf16* dy, int lddy, float* part) {
  extern __shared__ float sh[];
  float* ca = sh;
  float* cb = sh + s.c;
  const int n = blockIdx.y, chunk = blockIdx.x;
  for (int i = threadIdx.x; i < 2 * s.c; i += blockDim.x) sh[i] = 0.0f;
  __syncthreads();
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  if (r0 < s.R) {
    float gm[8], bt[8], mu[8], rs[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = cg * 8 + i, g = c / s.cpg;
      gm[i] = gamma[c];
      bt[i] = beta[c];
      mu[i] = stats[((long)n * s.groups + g) * 2];
      rs[i] = stats[((long)n * s.groups + g) * 2 + 1];
    }
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
    for (int row = rbeg + r0; row < rend; row += s.R) {
      float xh[8], gdy[8];
      gn_bwd_elem(s, n, row, cg, mu, rs, gm, bt, silu, dy, lddy, xh, gdy);
#pragma unroll
      for (int i = 0; i < 8; ++i) { a[i] += gdy[i]; b[i] += gdy[i] * xh[i]; }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      atomicAdd(&ca[cg * 8 + i], a[i]);
      atomicAdd(&cb[cg * 8 + i], b[i]);
    }
  }
  __syncthreads();
  for (int g = threadIdx.x; g < s.groups; g += blockDim.x) {
    float ta = 0.0f, tb = 0.0f;
    for (int k = 0; k < s.cpg; ++k) { ta += ca[g * s.cpg + k]; tb += cb[g * s.cpg + k]; }
    float* dst = part + (((long)n * s.nchunk + chunk) * s.groups + g) * 2;
    dst[0] = ta;
    dst[1] = tb;
  }
}

__global__ void gn_bwd_apply_kernel(GNShape s, const float* stats, const float* gamma, const float* beta, int silu,
                                    const bf16* dy, int lddy, const float* part, bf16* dx, int lddx,
                                    const bf16* add1, int ldadd1, const bf16* add2, int ldadd2) {
  __shared__ float ma[64], mb[64];
  const int n = blockIdx.y, chunk = blockIdx.x;
  for (int g = threadIdx.x; g < s.groups; g += blockDim.x) {
    double ta = 0.0, tb = 0.0;
    for (int k = 0; k < s.nchunk; ++k) {
      const float* src = part + (((long)n * s.nchunk + k) * s.groups + g) * 2;
      ta += src[0];
      tb += src[1];
    }
    const double cnt = (double)s.hw * s.cpg;
    ma[g] = (float)(ta / cnt);
    mb[g] = (float)(tb / cnt);
  }
  __syncthreads();
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  if (r0 >= s.R) return;
  float gm[8], bt[8], mu[8], rs[8], a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = cg * 8 + i, g = c / s.cpg;
    gm[i] = gamma[c];
    bt[i] = beta[c];
    mu[i] = stats[((long)n * s.groups + g) * 2];
    rs[i] = stats[((long)n * s.groups + g) * 2 + 1];
    a[i] = ma[g];
    b[i] = mb[g];
  }
  const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
  for (int row = rbeg + r0; row < rend; row += s.R) {
    float xh[8], gdy[8], out[8];
    gn_bwd_elem(s, n, row, cg, mu, rs, gm, bt, silu, dy, lddy, xh, gdy);
    const long pix = (long)n * s.hw + row;
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = rs[i] * (gdy[i] - a[i] - xh[i] * b[i]);
    if (add1) {
      float e[8];
      load8(add1 + pix * ldadd1 + cg * 8, e);
#pragma unroll
      for (int i = 0; i < 8; ++i) out[i] = (float)(bf16)out[i] + e[i];
    }
    if (add2) {
      float e[8];
      load8(add2 + pix * ldadd2 + cg * 8, e);
#pragma unroll
      for (int i = 0; i < 8; ++i) out[i] = (float)(bf16)out[i] + e[i];
    }
    store8(dx + pix * lddx + cg * 8, out);
  }
}

bool gn_make_shape(GNShape& s, const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c,
                   int groups) {
  if (!x || nb <= 0 || hw <= 0 || c <= 0 || groups <= 0 || groups > 64) return false;
  if (c % groups != 0 || c % 8 != 0) return false;
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
  // aim for >= ~64 rows per block but enough blocks to cover the chip
  int target_blocks = max(1, 512 / nb);
  s.rows_per_chunk = max(s.R, (hw + target_blocks - 1) / target_blocks);
  s.rows_per_chunk = ((s.rows_per_chunk + s.R - 1) / s.R) * s.R;
  s.nchunk = (hw + s.rows_per_chunk - 1) / s.rows_per_chunk;
  return true;
}

}  // namespace

extern "C" long long dc_groupnorm_ws_bytes(int nb, int hw, int c, int groups) {
  GNShape s;
  static const bf16 dummy[8] = {};
  if (!gn_make_shape(s, dummy, c, nullptr, 0, 0, nb, hw, c, groups)) return -1;
  return (long long)nb * s.nchunk * groups * 2 * sizeof(float);
}

extern "C" int dc_groupnorm_fwd(const void* x, int ldx, const void* x2, int ldx2, int c1, int nb, int hw, int c,
                                int groups, float eps, const float* gamma, const float* beta, int silu, void* y,
                                int ldy, float* stats, float* ws, void* stream) {
  GNShape s;
  if (!gn_make_shape(s, x, ldx, x2, ldx2, c1, nb, hw, c, groups) || !y || !gamma || !beta || !ws) return DC_ERR_ARG;
  if (ldy % 8) return DC_ERR_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  const int threads = s.cgs * s.R;
  dim3 grid(s.nchunk, nb);
  hipLaunchKernelGGL(gn_stats_kernel, grid, dim3(threads), 2 * c * sizeof(float), st, s, ws);
  hipLaunchKernelGGL(gn_apply_kernel, grid, dim3(threads), 0, st, s, ws, eps, gamma, beta, silu, (bf16*)y, ldy,
                     stats);
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
  const int threads = s.cgs * s.R;
  dim3 grid(s.nchunk, nb);
  hipLaunchKernelGGL(gn_bwd_stats_kernel, grid, dim3(threads), 2 * c * sizeof(float), st, s, stats, gamma, beta,
                     silu, (const bf16*)dy, lddy, ws);
  hipLaunchKernelGGL(gn_bwd_apply_kernel, grid, dim3(threads), 0, st, s, stats, gamma, beta, silu, (const bf16*)dy,
                     lddy, ws, (bf16*)dx, lddx, (const bf16*)add1, ldadd1, (const bf16*)add2, ldadd2);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// ---------------------------------------------------------------- LayerNorm (one wave per row)
namespace {

template <int MAXV>
__global__ void ln_fwd_kernel(const bf16* x, int ldx, long rows, int c, float eps, const float* gamma,
                              const float* beta, bf16* y, int ldy, float* stats) {
  const long row = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = c >> 3;
  float v[MAXV][8];
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      load8(x + row * ldx + vi * 8, v[k]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[k][i];
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
      for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mu) * rs * gamma[vi * 8 + i] + beta[vi * 8 + i];
      store8(y + row * ldy + vi * 8, o);
    }
  }
  if (lane == 0 && stats) {
    stats[row * 2] = mu;
    stats[row * 2 + 1] = rs;
  }
}

template <int MAXV>
__global__ void ln_bwd_kernel(const bf16* x, int ldx, long rows, int c, const float* gamma, const float* stats,
                              const bf16* dy, int lddy, bf16* dx, int lddx, const bf16* add, int ldadd) {
  const long row = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = c >> 3;
  const float mu = stats[row * 2], rs = stats[row * 2 + 1];
  float xh[MAXV][8], g[MAXV][8];
  float sa = 0.0f, sb = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      float f[8], d[8];
      load8(x + row * ldx + vi * 8, f);
      load8(dy + row * lddy + vi * 8, d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[k][i] = (f[i] - mu) * rs;
        g[k][i] = d[i] * gamma[vi * 8 + i];
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
        float e[8];
        load8(add + row * ldadd + vi * 8, e);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (float)(bf16)o[i] + e[i];
      }
      store8(dx + row * lddx + vi * 8, o);
    }
  }
}

}  // namespace

extern "C" int dc_layernorm_fwd(const void* x, int ldx, long long rows, int c, float eps, const float* gamma,
                                const float* beta, void* y, int ldy, float* stats, void* stream) {
  if (!x || !y || !gamma || !beta || rows <= 0 || c <= 0 || c % 8 || c > 2048 * 8) return DC_ERR_ARG;
  if (ldx % 8 || ldy % 8) return DC_ERR_ALIGN;
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
  if (!x || !dy || !dx || !gamma || !stats || rows <= 0 || c <= 0 || c % 8) return DC_ERR_ARG;
  if (ldx % 8 || lddy % 8 || lddx % 8 || (add && ldadd % 8)) return DC_ERR_ALIGN;
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

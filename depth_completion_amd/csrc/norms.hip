// GroupNorm(+SiLU) and LayerNorm forward / backward on NHWC rows (gfx950).
//
// GroupNorm (diffusers ResnetBlock2D norm1/norm2 + SiLU, Transformer2DModel.norm, conv_norm_out),
// three launches, all reductions in a fixed order (bitwise reproducible run to run):
//   stats     per (frame, pixel-chunk) block: 8 channels per thread in registers over its rows,
//             rows folded through LDS, channels folded into group partials -> slab [nb][nchunk][G][2]
//   finalize  one block per frame, one wave per group: fold the chunk partials (fp64) -> mean, rstd
//   apply     elementwise normalise (+ SiLU), 16 B per lane
// Backward: the same with (sum gamma*dy', sum gamma*dy'*xhat) and dx = rstd*(g*dy' - a - xhat*b).
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
  int apply_rows;  // rows per block of the elementwise passes
  int cgs, R;  // colgroups (c/8) and parallel rows per block
};

__device__ __forceinline__ void gn_load8(const GNShape& s, int n, int row, int c, float* f) {
  const long pix = (long)n * s.hw + row;
  const bf16* src = (c < s.c1) ? (s.x + pix * s.ldx + c) : (s.x2 + pix * s.ldx2 + (c - s.c1));
  load8(src, f);
}

// fold per-thread channel partials (a, b)[8] across the R row-lanes, then into group partials
__device__ void gn_block_fold(const GNShape& s, const float* a, const float* b, float* sh, float* out) {
  // sh: [2][R][c] floats
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  const bool active = r0 < s.R;
  float* sa = sh;
  float* sb = sh + s.R * s.c;
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
    for (int r = 0; r < s.R; ++r) { ta += sa[r * s.c + ch]; tb += sb[r * s.c + ch]; }
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

__global__ void gn_stats_kernel(GNShape s, float* part) {
  extern __shared__ float sh[];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < s.R) {
    const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
    for (int row = rbeg + r0; row < rend; row += s.R) {
      float f[8];
      gn_load8(s, n, row, cg * 8, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) { a[i] += f[i]; b[i] += f[i] * f[i]; }
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
    if (lane == 0) {
      float* dst = out + ((long)n * s.groups + g) * 2;
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
  }
}

// Elementwise passes: block (chunk, frame) with the stats kernel's thread layout -- each thread keeps
// one 8-channel group (cg = tid % cgs) over rows r0, r0 + R, ... -- so the per-channel coefficients
// are computed once per thread and the row loop carries no divisions.
__global__ void gn_apply_kernel(GNShape s, const float* stats, const float* gamma, const float* beta, int silu,
                                bf16* y, int ldy) {
  const int n = blockIdx.y;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  if (r0 >= s.R) return;
  float mu[8], rs[8], ga[8], be[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k, g = c / s.cpg;
    mu[k] = stats[((long)n * s.groups + g) * 2];
    rs[k] = stats[((long)n * s.groups + g) * 2 + 1];
    ga[k] = gamma[c];
    be[k] = beta[c];
  }
  const int rbeg = blockIdx.x * s.apply_rows, rend = min(s.hw, rbeg + s.apply_rows);
  for (int row = rbeg + r0; row < rend; row += s.R) {
    float f[8];
    gn_load8(s, n, row, cg * 8, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = (f[k] - mu[k]) * rs[k] * ga[k] + be[k];
      if (silu) v = silu_f((float)(bf16)v);
      f[k] = v;
    }
    store8(y + ((long)n * s.hw + row) * ldy + cg * 8, f);
  }
}

// dy' = dy * silu'(y) (y = gn(x) rounded to bf16, dy' rounded to bf16), as autograd does on bf16
__device__ __forceinline__ void gn_bwd_elem(const GNShape& s, int n, int row, int cg, const float* stats,
                                            const float* gamma, const float* beta, int silu, const bf16* dy,
                                            int lddy, float* xh, float* gdy, float* rsv) {
  float f[8], d[8];
  gn_load8(s, n, row, cg * 8, f);
  load8(dy + ((long)n * s.hw + row) * lddy + cg * 8, d);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = cg * 8 + i, g = c / s.cpg;
    const float mu = stats[((long)n * s.groups + g) * 2], rs = stats[((long)n * s.groups + g) * 2 + 1];
    const float xhat = (f[i] - mu) * rs;
    float dd = d[i];
    if (silu) {
      const float yv = (float)(bf16)(xhat * gamma[c] + beta[c]);
      dd = (float)(bf16)(dd * silu_grad(yv));
    }
    xh[i] = xhat;
    gdy[i] = dd * gamma[c];
    rsv[i] = rs;
  }
}

__global__ void gn_bwd_stats_kernel(GNShape s, const float* stats, const float* gamma, const float* beta, int silu,
                                    const bf16* dy, int lddy, float* part) {
  extern __shared__ float sh[];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < s.R) {
    const int rbeg = chunk * s.rows_per_chunk, rend = min(s.hw, rbeg + s.rows_per_chunk);
    for (int row = rbeg + r0; row < rend; row += s.R) {
      float xh[8], gdy[8], rs[8];
      gn_bwd_elem(s, n, row, cg, stats, gamma, beta, silu, dy, lddy, xh, gdy, rs);
#pragma unroll
      for (int i = 0; i < 8; ++i) { a[i] += gdy[i]; b[i] += gdy[i] * xh[i]; }
    }
  }
  gn_block_fold(s, a, b, sh, part + ((long)n * s.nchunk + chunk) * s.groups * 2);
}

__global__ void gn_bwd_apply_kernel(GNShape s, const float* stats, const float* gamma, const float* beta, int silu,
                                    const bf16* dy, int lddy, const float* ab, bf16* dx, int lddx,
                                    const bf16* add1, int ldadd1, const bf16* add2, int ldadd2) {
  const int n = blockIdx.y;
  const int cg = threadIdx.x % s.cgs, r0 = threadIdx.x / s.cgs;
  if (r0 >= s.R) return;
  float mu[8], rs[8], ga[8], be[8], ma[8], mb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k, g = c / s.cpg;
    mu[k] = stats[((long)n * s.groups + g) * 2];
    rs[k] = stats[((long)n * s.groups + g) * 2 + 1];
    ma[k] = ab[((long)n * s.groups + g) * 2];
    mb[k] = ab[((long)n * s.groups + g) * 2 + 1];
    ga[k] = gamma[c];
    be[k] = beta[c];
  }
  const int rbeg = blockIdx.x * s.apply_rows, rend = min(s.hw, rbeg + s.apply_rows);
  for (int row = rbeg + r0; row < rend; row += s.R) {
    const long pix = (long)n * s.hw + row;
    float f[8], d[8], out[8];
    gn_load8(s, n, row, cg * 8, f);
    load8(dy + pix * lddy + cg * 8, d);
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
    if (add1) {
      float e[8];
      load8(add1 + pix * ldadd1 + cg * 8, e);
#pragma unroll
      for (int k = 0; k < 8; ++k) out[k] = (float)(bf16)out[k] + e[k];
    }
    if (add2) {
      float e[8];
      load8(add2 + pix * ldadd2 + cg * 8, e);
#pragma unroll
      for (int k = 0; k < 8; ++k) out[k] = (float)(bf16)out[k] + e[k];
    }
    store8(dx + pix * lddx + cg * 8, out);
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
  // ~256-512 blocks over the whole launch, each at least R rows
  const int target_blocks = max(1, 384 / nb);
  s.rows_per_chunk = max(s.R, (hw + target_blocks - 1) / target_blocks);
  s.rows_per_chunk = ((s.rows_per_chunk + s.R - 1) / s.R) * s.R;
  s.nchunk = (hw + s.rows_per_chunk - 1) / s.rows_per_chunk;
  // elementwise passes: ~1024 blocks over the launch, at least R and at most 64 rows per block
  const int bpf = max(1, 1024 / nb);
  s.apply_rows = min(64, max(s.R, (hw + bpf - 1) / bpf));
  s.apply_rows = ((s.apply_rows + s.R - 1) / s.R) * s.R;
  return true;
}

// workspace layout: [partials nb*nchunk*G*2][ab nb*G*2]
inline long gn_part_floats(const GNShape& s) { return (long)s.nb * s.nchunk * s.groups * 2; }

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
  const int threads = s.cgs * s.R;
  const size_t lds = 2 * (size_t)s.R * s.c * sizeof(float);
  hipLaunchKernelGGL(gn_stats_kernel, dim3(s.nchunk, nb), dim3(threads), lds, st, s, ws);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((groups + 3) / 4, nb), dim3(256), 0, st, s, ws, eps, 0, stats);
  const dim3 agrid((hw + s.apply_rows - 1) / s.apply_rows, nb);
  hipLaunchKernelGGL(gn_apply_kernel, agrid, dim3(threads), 0, st, s, stats, gamma, beta, silu, (bf16*)y, ldy);
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
  const size_t lds = 2 * (size_t)s.R * s.c * sizeof(float);
  float* ab = ws + gn_part_floats(s);
  hipLaunchKernelGGL(gn_bwd_stats_kernel, dim3(s.nchunk, nb), dim3(threads), lds, st, s, stats, gamma, beta, silu,
                     (const bf16*)dy, lddy, ws);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((groups + 3) / 4, nb), dim3(256), 0, st, s, ws, 0.0f, 1, ab);
  const dim3 agrid((hw + s.apply_rows - 1) / s.apply_rows, nb);
  hipLaunchKernelGGL(gn_bwd_apply_kernel, agrid, dim3(threads), 0, st, s, stats, gamma, beta, silu,
                     (const bf16*)dy, lddy, ab, (bf16*)dx, lddx, (const bf16*)add1, ldadd1, (const bf16*)add2,
                     ldadd2);
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

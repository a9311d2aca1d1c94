// Memory-bound helpers of the hot path (gfx950): GEGLU fwd/bwd, nearest-upsample adjoint,
// TAESD latent clamp fwd/bwd, SiLU, image preprocessing (uint8 NCHW -> bf16 NHWC, antialiased
// bilinear resize, replicate pad) and layout conversions at the API boundary.
// All bf16 traffic is 16 B per lane where the layout allows (Guideline 13).
#include "common.h"
#include "../../include/dcamd.h"

namespace {

// f: [rows][2c] = (h | g) ; y = h * gelu(g)
__global__ void geglu_fwd_kernel(const bf16* f, int ldf, long rows, int c, bf16* y, int ldy) {
  const int cg = c / 8;
  const long total = rows * cg;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cg;
    const int col = (int)(i - r * cg) * 8;
    float h[8], g[8], o[8];
    load8(f + r * ldf + col, h);
    load8(f + r * ldf + c + col, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = h[k] * (float)(bf16)gelu_f(g[k]);
    store8(y + r * ldy + col, o);
  }
}

__global__ void geglu_bwd_kernel(const bf16* f, int ldf, long rows, int c, const bf16* dy, int lddy, bf16* df,
                                 int lddf) {
  const int cg = c / 8;
  const long total = rows * cg;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cg;
    const int col = (int)(i - r * cg) * 8;
    float h[8], g[8], d[8], dh[8], dg[8];
    load8(f + r * ldf + col, h);
    load8(f + r * ldf + c + col, g);
    load8(dy + r * lddy + col, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dh[k] = d[k] * (float)(bf16)gelu_f(g[k]);
      const float dgel = (float)(bf16)(d[k] * h[k]);
      dg[k] = dgel * gelu_grad(g[k]);
    }
    store8(df + r * lddf + col, dh);
    store8(df + r * lddf + c + col, dg);
  }
}

// nearest-upsample adjoint: dlo[Y][X] = sum over hi pixels (y,x) with floor(y*hlo/hhi)==Y, floor(x*wlo/whi)==X
__global__ void upsample_adjoint_kernel(const bf16* dhi, int ldhi, int nb, int hhi, int whi, int c, int hlo, int wlo,
                                        bf16* dlo, int ldlo, const bf16* mask, int ldmask) {
  const int cg = c / 8;
  const long total = (long)nb * hlo * wlo * cg;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int g = (int)(i % cg);
    const long pix = i / cg;
    const int X = (int)(pix % wlo);
    const long t = pix / wlo;
    const int Y = (int)(t % hlo);
    const int n = (int)(t / hlo);
    const int y0 = (int)(((long)Y * hhi + hlo - 1) / hlo), y1 = (int)(((long)(Y + 1) * hhi + hlo - 1) / hlo);
    const int x0 = (int)(((long)X * whi + wlo - 1) / wlo), x1 = (int)(((long)(X + 1) * whi + wlo - 1) / wlo);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (y1 - y0 == 2 && x1 - x0 == 2) {
      // the UNet's exact 2x: the four loads (and the mask's) in flight together, summed in the loop's order
      bf16x8 q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        q[j] = *reinterpret_cast<const bf16x8*>(dhi + (((long)n * hhi + y0 + (j >> 1)) * whi + x0 + (j & 1)) * ldhi +
                                                g * 8);
      bf16x8 mq;
      if (mask) mq = *reinterpret_cast<const bf16x8*>(mask + pix * ldmask + g * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += (float)q[j][k];
      if (mask) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = (float)mq[k] > 0.0f ? acc[k] : 0.0f;
      }
      store8(dlo + pix * ldlo + g * 8, acc);
      continue;
    }
    for (int y = y0; y < y1; ++y)
      for (int x = x0; x < x1; ++x) {
        float v[8];
        load8(dhi + (((long)n * hhi + y) * whi + x) * ldhi + g * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[k];
      }
    if (mask) {
      float mk[8];
      load8(mask + pix * ldmask + g * 8, mk);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = mk[k] > 0.0f ? acc[k] : 0.0f;
    }
    store8(dlo + pix * ldlo + g * 8, acc);
  }
}

// TAESD DecoderTiny input clamp: y = tanh(x/3)*3 ; x [P][ldx] (4 used), y [P][8] (4..7 zero)
__global__ void taesd_clamp_fwd_kernel(const bf16* x, int ldx, long P, bf16* y) {
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
    float o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = (float)(bf16)((float)x[p * ldx + k] / 3.0f);
      const float t = (float)(bf16)tanhf(a);
      o[k] = t * 3.0f;
      o[k + 4] = 0.0f;
    }
    store8(y + p * 8, o);
  }
}

// backward of tanh(x/3)*3 (bf16 autograd chain), then of x0 = sqrt(a)*x - sqrt(b)*v:
//   gx0 -> gx_direct = gx0*sqrt(a) (bf16), dv = -gx0*sqrt(b) (bf16, into dv[P][8], 4..7 zero)
__global__ void taesd_clamp_bwd_kernel(const bf16* x0, int ldx0, const bf16* dy, int lddy, long P, const float* coef,
                                       const int* step, bf16* gx_direct, bf16* dv) {
  // the first pixel's rows go out before the step's dependent coefficient reads (8-B vectors; clamped, skipped)
  long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  bf16x4 xr = *reinterpret_cast<const bf16x4*>(x0 + min(p, P - 1) * ldx0);
  bf16x4 dr = *reinterpret_cast<const bf16x4*>(dy + min(p, P - 1) * lddy);
  asm volatile("" ::: "memory");
  const float sa = coef[*step * 4 + 0], sb = coef[*step * 4 + 1];
  for (bool first = true; p < P; p += (long)gridDim.x * blockDim.x, first = false) {
    if (!first) {
      xr = *reinterpret_cast<const bf16x4*>(x0 + p * ldx0);
      dr = *reinterpret_cast<const bf16x4*>(dy + p * lddy);
    }
    float gd[8], vv[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = (float)(bf16)((float)xr[k] / 3.0f);
      const float t = (float)(bf16)tanhf(a);
      float g = (float)(bf16)((float)dr[k] * 3.0f);
      g = (float)(bf16)(g * (1.0f - t * t));
      g = (float)(bf16)(g / 3.0f);
      gd[k] = g * sa;
      vv[k] = -g * sb;
      gd[k + 4] = 0.0f;
      vv[k + 4] = 0.0f;
    }
    store8(gx_direct + p * 8, gd);
    store8(dv + p * 8, vv);
  }
}

__global__ void silu_kernel(const bf16* x, long n, bf16* y) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = (bf16)silu_f((float)x[i]);
}

// ---- image preprocessing (MarigoldImageProcessor.preprocess + EncoderTiny's x.add(1).div(2))
// u8 NCHW [nb][3][H][W] -> bf16 [nb][PH][PW][8] (channels 3..7 zero), with antialiased bilinear
// resize (H,W) -> (RH,RW) in the [-1,1] domain and replicate padding to (PH,PW).
__device__ __forceinline__ float aa_filter(float x) {
  x = fabsf(x);
  return x < 1.0f ? 1.0f - x : 0.0f;
}

__global__ void preprocess_kernel(const uint8_t* img, int nb, int H, int W, int RH, int RW, int PH, int PW,
                                  int encoder_input, bf16* out) {
  const long total = (long)nb * PH * PW;
  const float sh = (float)H / RH, sw = (float)W / RW;
  const float supy = sh >= 1.0f ? sh : 1.0f, supx = sw >= 1.0f ? sw : 1.0f;
  const float invy = sh >= 1.0f ? 1.0f / sh : 1.0f, invx = sw >= 1.0f ? 1.0f / sw : 1.0f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int px = (int)(i % PW);
    const long t = i / PW;
    const int py = (int)(t % PH);
    const int n = (int)(t / PH);
    const int oy = min(py, RH - 1), ox = min(px, RW - 1);  // replicate pad (bottom / right)
    float o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool identity = (RH == H && RW == W);
    for (int ch = 0; ch < 3; ++ch) {
      const uint8_t* plane = img + ((long)n * 3 + ch) * H * W;
      float v;
      if (identity) {
        v = (float)(bf16)((float)(bf16)((float)plane[(long)oy * W + ox] / 255.0f) * 2.0f - 1.0f);
      } else {
        const float cy = sh * (oy + 0.5f), cx = sw * (ox + 0.5f);
        const int ymin = max((int)(cy - supy + 0.5f), 0), ymax = min((int)(cy + supy + 0.5f), H);
        const int xmin = max((int)(cx - supx + 0.5f), 0), xmax = min((int)(cx + supx + 0.5f), W);
        float wy_tot = 0.0f, wx_tot = 0.0f;
        for (int y = ymin; y < ymax; ++y) wy_tot += aa_filter((y - cy + 0.5f) * invy);
        for (int x = xmin; x < xmax; ++x) wx_tot += aa_filter((x - cx + 0.5f) * invx);
        float acc = 0.0f;
        for (int y = ymin; y < ymax; ++y) {
          const float wy = aa_filter((y - cy + 0.5f) * invy) / wy_tot;
          float row = 0.0f;
          for (int x = xmin; x < xmax; ++x) {
            const float wx = aa_filter((x - cx + 0.5f) * invx) / wx_tot;
            const float pv = (float)(bf16)((float)(bf16)((float)plane[(long)y * W + x] / 255.0f) * 2.0f - 1.0f);
            row += wx * pv;
          }
          acc += wy * row;
        }
        v = (float)(bf16)acc;
      }
      if (encoder_input) v = (float)(bf16)((float)(bf16)(v + 1.0f) / 2.0f);
      o[ch] = v;
    }
    store8(out + i * 8, o);
  }
}

// NHWC [P][ldx] (first c channels) <-> NCHW [nb][c][hw]
__global__ void nhwc_to_nchw_kernel(const bf16* x, int ldx, int nb, long hw, int c, bf16* y) {
  const long total = (long)nb * hw * c;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i % hw;
    const long t = i / hw;
    const int ch = (int)(t % c);
    const long n = t / c;
    y[i] = x[(n * hw + p) * ldx + ch];
  }
}
__global__ void nchw_to_nhwc_kernel(const bf16* x, int nb, long hw, int c, bf16* y, int ldy) {
  const long total = (long)nb * hw * c;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i % hw;
    const long t = i / hw;
    const int ch = (int)(t % c);
    const long n = t / c;
    y[(n * hw + p) * ldy + ch] = x[i];
  }
}

inline dim3 grid_for(long n, int per_block = 256) {
  long b = (n + per_block - 1) / per_block;
  if (b > 65536) b = 65536;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

}  // namespace

extern "C" int dc_geglu_fwd(const void* f, int ldf, long long rows, int c, void* y, int ldy, void* stream) {
  if (!f || !y || rows <= 0 || c <= 0 || c % 8) return DC_ERR_ARG;
  if (ldf % 8 || ldy % 8) return DC_ERR_ALIGN;
  hipLaunchKernelGGL(geglu_fwd_kernel, grid_for(rows * (c / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)f,
                     ldf, (long)rows, c, (bf16*)y, ldy);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_geglu_bwd(const void* f, int ldf, long long rows, int c, const void* dy, int lddy, void* df, int lddf,
                            void* stream) {
  if (!f || !dy || !df || rows <= 0 || c <= 0 || c % 8) return DC_ERR_ARG;
  if (ldf % 8 || lddy % 8 || lddf % 8) return DC_ERR_ALIGN;
  hipLaunchKernelGGL(geglu_bwd_kernel, grid_for(rows * (c / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)f,
                     ldf, (long)rows, c, (const bf16*)dy, lddy, (bf16*)df, lddf);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_upsample_adjoint(const void* dhi, int ldhi, int nb, int hhi, int whi, int c, int hlo, int wlo,
                                   void* dlo, int ldlo, const void* mask, int ldmask, void* stream) {
  if (!dhi || !dlo || nb <= 0 || hhi < hlo || whi < wlo || hlo <= 0 || wlo <= 0 || c % 8) return DC_ERR_ARG;
  if (ldhi % 8 || ldlo % 8 || (mask && ldmask % 8)) return DC_ERR_ALIGN;
  hipLaunchKernelGGL(upsample_adjoint_kernel, grid_for((long)nb * hlo * wlo * (c / 8)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)dhi, ldhi, nb, hhi, whi, c, hlo, wlo, (bf16*)dlo, ldlo,
                     (const bf16*)mask, ldmask);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_taesd_clamp_fwd(const void* x, int ldx, long long pixels, void* y, void* stream) {
  if (!x || !y || pixels <= 0 || ldx < 4) return DC_ERR_ARG;
  hipLaunchKernelGGL(taesd_clamp_fwd_kernel, grid_for(pixels), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, ldx,
                     (long)pixels, (bf16*)y);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_taesd_clamp_bwd(const void* x0, int ldx0, const void* dy, int lddy, long long pixels,
                                  const float* coef, const int* step, void* gx_direct, void* dv, void* stream) {
  if (!x0 || !dy || !coef || !step || !gx_direct || !dv || pixels <= 0) return DC_ERR_ARG;
  if (ldx0 % 4 || lddy % 4 || ((uintptr_t)x0 & 7) || ((uintptr_t)dy & 7)) return DC_ERR_ALIGN;
  hipLaunchKernelGGL(taesd_clamp_bwd_kernel, grid_for(pixels), dim3(256), 0, (hipStream_t)stream, (const bf16*)x0,
                     ldx0, (const bf16*)dy, lddy, (long)pixels, coef, step, (bf16*)gx_direct, (bf16*)dv);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_silu(const void* x, long long n, void* y, void* stream) {
  if (!x || !y || n <= 0) return DC_ERR_ARG;
  hipLaunchKernelGGL(silu_kernel, grid_for(n), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (long)n, (bf16*)y);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_preprocess_image(const void* img_u8, int nb, int h, int w, int rh, int rw, int ph, int pw,
                                   int encoder_input, void* out, void* stream) {
  if (!img_u8 || !out || nb <= 0 || h <= 0 || w <= 0 || rh <= 0 || rw <= 0 || ph < rh || pw < rw) return DC_ERR_ARG;
  hipLaunchKernelGGL(preprocess_kernel, grid_for((long)nb * ph * pw), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)img_u8, nb, h, w, rh, rw, ph, pw, encoder_input, (bf16*)out);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_nhwc_to_nchw(const void* x, int ldx, int nb, long long hw, int c, void* y, void* stream) {
  if (!x || !y || nb <= 0 || hw <= 0 || c <= 0 || ldx < c) return DC_ERR_ARG;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, grid_for((long)nb * hw * c), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ldx, nb, (long)hw, c, (bf16*)y);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_nchw_to_nhwc(const void* x, int nb, long long hw, int c, void* y, int ldy, void* stream) {
  if (!x || !y || nb <= 0 || hw <= 0 || c <= 0 || ldy < c) return DC_ERR_ARG;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, grid_for((long)nb * hw * c), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, nb, (long)hw, c, (bf16*)y, ldy);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// The sparse-depth guidance of one guided DDIM step (marigold_dc.py:806-904) as fused gfx950 kernels.
//
//   dc_sparse_setup     once per call: compact LiDAR pixels (sparses > 0) per frame, sparse
//                       normalisation (marigold_dc.py:706-756), masked min/max of the guides
//                       (utils.py:89-138 as used by _affine_to_metric, marigold_dc.py:326)
//   dc_preview          Tweedie preview x0 = sqrt(a)x - sqrt(1-a)v, TAESD clamp input tanh(x0/3)*3,
//                       ||eps||, eps = sqrt(a)v + sqrt(1-a)x      (marigold_dc.py:813-826)
//   dc_sparse_loss      decode tail (x*2-1, channel mean, clip, (x+1)/2), bilinear resize at the
//                       sparse pixels only, learned affine + clamp, l1+l2 loss, its gradient
//                       scattered into the decoded-depth image, d(scale), d(shift)  (:829-877)
//   dc_decode_tail_bwd  gradient of the decode tail back to the TAESD decoder output
//   dc_latent_update    grad accumulation (+ KL term), ||eps||/||g|| rescale, Adam / SGD / Adagrad (bf16
//                       state for the latent, fp32 for scale/shift), DDIM prev-sample on the updated latent
//                       (:879-904)
//   dc_final_dense      final decode -> affine -> clamp -> metres (:969-985)
// Elementwise arithmetic mirrors PyTorch's op-by-op rounding (bf16 results of bf16 ops, fp32 for
// the affine/loss), so the only deviation from the reference is reduction order.
#include "common.h"
#include <stdlib.h>
#include "../../include/dcamd.h"

#pragma clang fp contract(off)

namespace {

constexpr int SETUP_THREADS = 1024;

__device__ __forceinline__ float proj_f(float v, int projection) {
  if (projection == 1) return logf(v);
  if (projection == 2) return log10f(v);
  return v;
}

__device__ float block_min(float v, float* scratch) {
  for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float t = l < nw ? scratch[l] : INFINITY;
  for (int o = 32; o >= 1; o >>= 1) t = fminf(t, __shfl_xor(t, o, 64));
  return t;
}
__device__ float block_max(float v, float* scratch) { return -block_min(-v, scratch); }

// params per frame: [0]=lo [1]=hi (metres) [2]=lo_p [3]=hi_p [4]=min_g [5]=max_g [6]=count
// [7]=projection + 4 inv (the depth space the loss compares in) + 8 nearest (interp_mode)
__global__ void sparse_setup_kernel(const float* sparse, int H, int W, int norm, float min_depth, float max_depth,
                                    const float* host_lohi, int projection, int inv, int interp, int* idx, float* gval,
                                    int* cnt, float* params) {
  __shared__ int wave_counts[SETUP_THREADS / 64];
  __shared__ float scratch[SETUP_THREADS / 64];
  __shared__ int base_sh;
  const int n = blockIdx.x;
  const long HW = (long)H * W;
  const float* sp = sparse + n * HW;
  int* ix = idx + n * HW;
  float* gv = gval + n * HW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float rmin = INFINITY, rmax = -INFINITY;
  // Compaction in pixel order: thread t owns the contiguous run [t R, (t + 1) R) (R = HW / threads, rounded up to 4
  // pixels for 16-B loads).  Pass 1 counts each run (and the masked min / max), one block scan gives every run its
  // output offset, pass 2 re-reads the run and writes its points -- two barriers in all, where a block-wide ballot per
  // 1024 pixels paid three barriers per step (~0.57 ms per C2 frame).
  const long R = ((HW + blockDim.x - 1) / blockDim.x + 3) & ~3L;
  const long r0 = min(HW, (long)threadIdx.x * R), r1 = min(HW, r0 + R);
  const bool vec = (HW & 3) == 0 && (((uintptr_t)sp) & 15) == 0;
  auto quad = [&](long p) __attribute__((always_inline)) {   // pixels p .. p + 3 of the run (0 beyond it)
    if (vec) return *reinterpret_cast<const float4*>(sp + p);
    float4 q;
    q.x = sp[p];
    q.y = p + 1 < r1 ? sp[p + 1] : 0.0f;
    q.z = p + 2 < r1 ? sp[p + 2] : 0.0f;
    q.w = p + 3 < r1 ? sp[p + 3] : 0.0f;
    return q;
  };
  int mine = 0;
#pragma unroll 4
  for (long p = r0; p < r1; p += 4) {
    const float4 q = quad(p);
    const float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (e[k] > 0.0f) {
        ++mine;
        rmin = fminf(rmin, e[k]);
        rmax = fmaxf(rmax, e[k]);
      }
  }
  // exclusive block scan of the run counts (wave scan by shuffles, then the wave totals)
  int incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wave_counts[w] = incl;
  __syncthreads();
  int off = incl - mine;
  for (int k = 0; k < w; ++k) off += wave_counts[k];
  if (threadIdx.x == blockDim.x - 1) base_sh = off + mine;
#pragma unroll 4
  for (long p = r0; p < r1; p += 4) {
    const float4 q = quad(p);
    const float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (e[k] > 0.0f) {
        ix[off] = (int)(p + k);
        gv[off] = e[k];
        ++off;
      }
  }
  __syncthreads();
  const int count = base_sh;
  (void)nw;
  rmin = block_min(rmin, scratch);
  rmax = block_max(rmax, scratch);
  float lo, hi;
  if (norm == 0) {           // const
    lo = min_depth;
    hi = max_depth;
  } else if (norm == 1) {    // minmax
    lo = rmin;
    hi = rmax;
  } else {                   // percentile: provided by the host (quantiles of the masked values)
    lo = host_lohi[2 * n];
    hi = host_lohi[2 * n + 1];
  }
  const float lo_c = lo, hi_c = hi;  // sparses.clamp(min=lo, max=hi) uses the un-clamped range
  if (norm != 0) {
    lo = fmaxf(lo, min_depth);
    hi = fminf(hi, max_depth);
  }
  float lo_p = proj_f(lo, projection), hi_p = proj_f(hi, projection);
  if (inv) {
    const float a = 1.0f / hi_p, b = 1.0f / lo_p;
    lo_p = a;
    hi_p = b;
  }
  float gmin = INFINITY, gmax = -INFINITY;
  __syncthreads();
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    float v = fminf(fmaxf(gv[k], lo_c), hi_c);
    v = proj_f(v, projection);
    if (inv) v = 1.0f / v;
    const float g = (v - lo_p) / (hi_p - lo_p);
    gv[k] = g;
    gmin = fminf(gmin, g);
    gmax = fmaxf(gmax, g);
  }
  gmin = block_min(gmin, scratch);
  gmax = block_max(gmax, scratch);
  if (threadIdx.x == 0) {
    cnt[n] = count;
    float* pr = params + n * 8;
    pr[0] = lo; pr[1] = hi; pr[2] = lo_p; pr[3] = hi_p; pr[4] = gmin; pr[5] = gmax;
    // the loss's depth space (DSpace) and the resize's interpolation (sample_affine)
    pr[6] = (float)count; pr[7] = (float)(projection + 4 * inv + 8 * interp);
  }
}

// coef table per step: [sqrt(a_t), sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev)]
__global__ void preview_kernel(const bf16* x8, const bf16* v, int hw, const float* coef, const int* step, bf16* x0,
                               bf16* tin, float* eps_norm) {
  __shared__ float scratch[16];
  const int n = blockIdx.x;
  // one block per frame (the norm below is a block sum): each thread's pixels are loaded kPf at a time, all of them
  // before the coefficients' dependent reads -- one pixel per round trip made this launch ~20 us at C2
  constexpr int kPf = 8;
  float ss = 0.0f;
  float sa = 0.0f, sb = 0.0f;
  for (int p0 = threadIdx.x; p0 < hw; p0 += kPf * blockDim.x) {
    bf16x8 xr[kPf], vr[kPf];
#pragma unroll
    for (int u = 0; u < kPf; ++u) {
      const long pix = (long)n * hw + min(p0 + u * (int)blockDim.x, hw - 1);
      xr[u] = *reinterpret_cast<const bf16x8*>(x8 + pix * 8);
      vr[u] = *reinterpret_cast<const bf16x8*>(v + pix * 8);
    }
    if (p0 == (int)threadIdx.x) {
      sa = coef[*step * 4 + 0];
      sb = coef[*step * 4 + 1];
    }
#pragma unroll
    for (int u = 0; u < kPf; ++u) {
      const int p = p0 + u * blockDim.x;
      if (p >= hw) continue;
      const long pix = (long)n * hw + p;
      float xo[8], to[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x = (float)xr[u][4 + k];
        const float vv = (float)vr[u][k];
        const float t1 = (float)(bf16)(sa * x), t2 = (float)(bf16)(sb * vv);
        const float xz = (float)(bf16)(t1 - t2);
        const float e = (float)(bf16)((float)(bf16)(sa * vv) + (float)(bf16)(sb * x));
        ss += e * e;
        xo[k] = xz;
        xo[k + 4] = 0.0f;
        const float a = (float)(bf16)(xz / 3.0f);
        to[k] = (float)(bf16)((float)(bf16)tanhf(a) * 3.0f);
        to[k + 4] = 0.0f;
      }
      store8(x0 + pix * 8, xo);
      store8(tin + pix * 8, to);
    }
  }
  const float tot = block_sum(ss, scratch);
  if (threadIdx.x == 0) eps_norm[n] = (float)(bf16)sqrtf(tot);
}

// decoded-affine value A at processing-res pixel (y, x): decode tail of TAESD output `out` [PH*PW][ldo]
__device__ __forceinline__ float decode_tail(const bf16* out, int ldo, long pix) {
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c) s += (float)(bf16)((float)(bf16)((float)out[pix * ldo + c] * 2.0f) - 1.0f);
  const float mean = (float)(bf16)(s * (1.0f / 3.0f));
  const float cl = fminf(fmaxf(mean, -1.0f), 1.0f);
  return (float)(bf16)((float)(bf16)(cl + 1.0f) / 2.0f);
}

struct Taps {
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
};
// upsample_bilinear2d (align_corners=False, no antialias) source taps for output (y,x): in (RH,RW) -> out (H,W)
__device__ __forceinline__ Taps bilinear_taps(int y, int x, int RH, int RW, int H, int W) {
  Taps t;
  const float rh = (float)RH / H, rw = (float)RW / W;
  float sy = rh * (y + 0.5f) - 0.5f;
  sy = sy < 0.0f ? 0.0f : sy;
  float sx = rw * (x + 0.5f) - 0.5f;
  sx = sx < 0.0f ? 0.0f : sx;
  t.y0 = (int)sy;
  t.x0 = (int)sx;
  t.y1 = t.y0 + ((t.y0 < RH - 1) ? 1 : 0);
  t.x1 = t.x0 + ((t.x0 < RW - 1) ? 1 : 0);
  t.ly1 = sy - t.y0;
  t.ly0 = 1.0f - t.ly1;
  t.lx1 = sx - t.x0;
  t.lx0 = 1.0f - t.lx1;
  return t;
}

// upsample_nearest2d source index (torch: identity at equal size, >> 1 at exactly 2x, else
// min(floor(dst * (in / out)), in - 1) in fp32)
__device__ __forceinline__ int nearest_src(int dst, int in, int out) {
  if (in == out) return dst;
  if (out == 2 * in) return dst >> 1;
  const float scale = (float)in / (float)out;
  const int s = (int)floorf((float)dst * scale);
  return s < in - 1 ? s : in - 1;
}

// interpolation of _latent_to_affine's resize (marigold_dc.py:366-370): params[7] bit 3 = nearest
__device__ __forceinline__ int interp_nearest(const float* pr) { return ((int)pr[7] >> 3) & 1; }

__device__ __forceinline__ float sample_affine(const bf16* out, int ldo, int n, int PH, int PW, int RH, int RW, int H,
                                               int W, int y, int x, Taps& t, int nearest) {
  const long base = (long)n * PH * PW;
  if (nearest) {
    t.y0 = t.y1 = nearest_src(y, RH, H);
    t.x0 = t.x1 = nearest_src(x, RW, W);
    t.ly0 = t.lx0 = 1.0f;
    t.ly1 = t.lx1 = 0.0f;
    return decode_tail(out, ldo, base + (long)t.y0 * PW + t.x0);
  }
  if (RH == H && RW == W) {
    t.y0 = t.y1 = y;
    t.x0 = t.x1 = x;
    t.ly0 = t.lx0 = 1.0f;
    t.ly1 = t.lx1 = 0.0f;
    return decode_tail(out, ldo, base + (long)y * PW + x);
  }
  t = bilinear_taps(y, x, RH, RW, H, W);
  const float a00 = decode_tail(out, ldo, base + (long)t.y0 * PW + t.x0);
  const float a01 = decode_tail(out, ldo, base + (long)t.y0 * PW + t.x1);
  const float a10 = decode_tail(out, ldo, base + (long)t.y1 * PW + t.x0);
  const float a11 = decode_tail(out, ldo, base + (long)t.y1 * PW + t.x1);
  const float v = t.ly0 * (t.lx0 * a00 + t.lx1 * a01) + t.ly1 * (t.lx0 * a10 + t.lx1 * a11);
  return (float)(bf16)v;
}

// Depth space of the loss (marigold_dc.py:843-860, 930-948): the clamped normalised depth G goes back to
// metres, through the projection (log / log10) and / or the inverse, and is renormalised with the
// projected bounds; returns that value and dN/dG.  The identity for linear without inverse.
struct DSpace {
  int proj, inv;
  float lo, hi, lo_p, hi_p;
  __device__ explicit DSpace(const float* pr) {
    const int code = (int)pr[7];
    proj = code & 3;
    inv = (code >> 2) & 1;
    lo = pr[0]; hi = pr[1]; lo_p = pr[2]; hi_p = pr[3];
  }
  __device__ float operator()(float G, float& dNdG) const {
    if (proj == 0 && !inv) {
      dNdG = 1.0f;
      return G;
    }
    const float span = hi - lo;
    const float D = G * span + lo;
    float P = D, dP = 1.0f;
    if (proj == 1) { P = logf(D); dP = 1.0f / D; }
    else if (proj == 2) { P = log10f(D); dP = 1.0f / (D * 2.302585093f); }
    float Q = P, dQ = 1.0f;
    if (inv) { Q = 1.0f / P; dQ = -1.0f / (P * P); }
    const float den = hi_p - lo_p;
    dNdG = (dQ * dP * span) / den;
    return (Q - lo_p) / den;
  }
};

// one block per frame.  affine[n*2] = scale, affine[n*2+1] = shift (fp32 trainables)
__global__ void sparse_loss_kernel(const bf16* out, int ldo, int PH, int PW, int RH, int RW, int H, int W,
                                   const int* idx, const float* gval, const int* cnt, const float* params,
                                   const float* affine, float* dA, float* daff_grad, float* loss) {
  __shared__ float scratch[16];
  const int n = blockIdx.x;
  const long HW = (long)H * W;
  // the thread's first point index and guide go out with the count and the parameters (a clamped slot, used only
  // when it is a point): not after the count, one round trip less
  const long k0 = min((long)threadIdx.x, HW - 1);
  const int p0 = idx[n * HW + k0];
  const float g0 = gval[n * HW + k0];
  const int count = cnt[n];
  const float* pr = params + n * 8;
  const float gmin = pr[4], gmax = pr[5];
  const float s = affine[n * 2], sh = affine[n * 2 + 1];
  const float A1 = s * s;
  const float B = A1 * (gmax - gmin);
  const float E = (sh * sh) * gmin;
  const float inv_cnt = 1.0f / (float)count;
  float sum_db = 0.0f, sum_de = 0.0f, lsum = 0.0f;
  float* dAn = dA + (long)n * PH * PW;
  const DSpace ds(pr);
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    const bool first = k == (int)threadIdx.x;
    const int p = first ? p0 : idx[n * HW + k];
    const int y = p / W, x = p - (p / W) * W;
    Taps t;
    const float aff = sample_affine(out, ldo, n, PH, PW, RH, RW, H, W, y, x, t, interp_nearest(pr));
    const float F = B * aff + E;
    float dNdG;
    const float Nv = ds(fminf(fmaxf(F, 0.0f), 1.0f), dNdG);
    const float r = Nv - (first ? g0 : gval[n * HW + k]);
    lsum += fabsf(r) * inv_cnt + (r * r) * inv_cnt;
    const float sg = (r > 0.0f) ? 1.0f : ((r < 0.0f) ? -1.0f : 0.0f);
    const float dG = (sg * inv_cnt + 2.0f * r * inv_cnt) * dNdG;
    const float dF = (F >= 0.0f && F <= 1.0f) ? dG : 0.0f;
    sum_db += dF * aff;
    sum_de += dF;
    const float dff = (float)(bf16)(dF * B);
    if (t.ly1 == 0.0f && t.lx1 == 0.0f && t.y0 == t.y1 && t.x0 == t.x1) {
      atomicAdd(&dAn[(long)t.y0 * PW + t.x0], dff);
    } else {
      atomicAdd(&dAn[(long)t.y0 * PW + t.x0], t.ly0 * t.lx0 * dff);
      atomicAdd(&dAn[(long)t.y0 * PW + t.x1], t.ly0 * t.lx1 * dff);
      atomicAdd(&dAn[(long)t.y1 * PW + t.x0], t.ly1 * t.lx0 * dff);
      atomicAdd(&dAn[(long)t.y1 * PW + t.x1], t.ly1 * t.lx1 * dff);
    }
  }
  const float db = block_sum(sum_db, scratch);
  __syncthreads();
  const float de = block_sum(sum_de, scratch);
  __syncthreads();
  const float ls = block_sum(lsum, scratch);
  if (threadIdx.x == 0) {
    const float dA1 = db * (gmax - gmin);
    daff_grad[n * 2] = dA1 * (2.0f * s);
    daff_grad[n * 2 + 1] = (de * gmin) * (2.0f * sh);
    loss[n] = ls;
  }
}

// dA (fp32, [nb][PH][PW]) -> gradient of the TAESD decoder output (bf16 [P][8], channels 0..2)
__global__ void decode_tail_bwd_kernel(const bf16* out, int ldo, const float* dA, int nb, int PH, int PW, int RH,
                                       int RW, bf16* dout) {
  const long total = (long)nb * PH * PW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % PW);
    const int y = (int)((i / PW) % PH);
    float g = 0.0f;
    if (y < RH && x < RW) {
      g = (float)(bf16)dA[i];
      if (g != 0.0f) {
        g = (float)(bf16)(g / 2.0f);
        float s = 0.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) s += (float)(bf16)((float)(bf16)((float)out[i * ldo + c] * 2.0f) - 1.0f);
        const float mean = (float)(bf16)(s * (1.0f / 3.0f));
        g = (mean >= -1.0f && mean <= 1.0f) ? g : 0.0f;
        g = (float)(bf16)(g / 3.0f);
        g = (float)(bf16)(g * 2.0f);
      }
    }
    float o[8] = {g, g, g, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    store8(dout + i * 8, o);
  }
}

// adam_tab per step: [step_size = lr_lat/bc1, bc2_sqrt, step_size_aff = lr_aff/bc1, unused]
// KL term of compute_loss (kld=True, marigold_dc.py:239-243 -> utils.kld_stdnorm, utils.py:28-86) on the
// bf16 latent x, per frame over M = 4 hw elements: mode 1 "simple" mean(x^2) -> 2x/M; mode 2 "strict"
// 0.5 (mu^2 + var - log(var + eps) - 1) -> mu/M + (x - mu)/M (1 - 1/(var + eps)), eps = bf16 eps; times
// kld_weight, as autograd forms it in bf16.
struct Kld {
  int mode;
  float w, mu, var_eps, inv_m;
  __device__ float grad(float x) const {
    if (mode == 1) return (float)(bf16)((float)(bf16)((float)(bf16)w * inv_m) * (2.0f * x));
    const float d = (float)(bf16)((x - mu) * inv_m);
    return (float)(bf16)(w * (float)(bf16)(mu * inv_m + d * (1.0f - 1.0f / var_eps)));
  }
};

// Per-element second pass of the latent update (rescaled gradient g): Adam / SGD / Adagrad with torch's
// bf16 rounding per op, then the DDIM prev-sample with the pre-update v.
struct UpdCtx {
  float sa, sb, sap, sbp, step_size, bc2s, step_aff;
  int opt;
};
// the arithmetic on values (x: the latent, vm: v, g: the rescaled gradient; m / vv: the optimiser state, updated in
// place as the rule writes it): returns the new latent
__device__ __forceinline__ float latent_elem_core(const UpdCtx& u, float x, float vm, float g, float& m, float& vv) {
  const float beta1w = 0.1f, beta2 = 0.999f, one_m_b2 = 0.001f, eps = 1e-8f;
  const float sa = u.sa, sb = u.sb, sap = u.sap, sbp = u.sbp, step_size = u.step_size, bc2s = u.bc2s;
  const int opt = u.opt;
  float xp;
  if (opt == 0) {
    m = (float)(bf16)(m + beta1w * (g - m));
    vv = (float)(bf16)(vv * beta2);
    vv = (float)(bf16)(vv + one_m_b2 * g * g);
    float den = (float)(bf16)sqrtf(vv);
    den = (float)(bf16)(den / bc2s);
    den = (float)(bf16)(den + eps);
    xp = (float)(bf16)(x + (-step_size) * (m / den));
  } else if (opt == 1) {
    xp = (float)(bf16)(x + (-step_size) * g);
  } else {
    const float sum = (float)(bf16)(m + g * g);
    m = sum;
    const float sd = (float)(bf16)((float)(bf16)sqrtf(sum) + 1e-10f);
    xp = (float)(bf16)(x + (-step_size) * (g / sd));
  }
  const float x0 = (float)(bf16)((float)(bf16)(sa * xp) - (float)(bf16)(sb * vm));
  const float ep = (float)(bf16)((float)(bf16)(sa * vm) + (float)(bf16)(sb * xp));
  const float dir = (float)(bf16)(sbp * ep);
  return (float)(bf16)((float)(bf16)(sap * x0) + dir);
}
__device__ __forceinline__ void latent_elem_update(const UpdCtx& u, bf16* x8, const bf16* v, bf16* m_lat, bf16* v_lat,
                                                   long pix, int k, float g) {
  const long e = pix * 4 + k;
  float m = u.opt == 1 ? 0.0f : (float)m_lat[e];
  float vv = u.opt == 0 ? (float)v_lat[e] : 0.0f;
  const float prev = latent_elem_core(u, (float)x8[pix * 8 + 4 + k], (float)v[pix * 8 + k], g, m, vv);
  if (u.opt != 1) m_lat[e] = (bf16)m;
  if (u.opt == 0) v_lat[e] = (bf16)vv;
  x8[pix * 8 + 4 + k] = (bf16)prev;
}

// the same rule on scale (j = 0) / shift (j = 1), fp32 state
__device__ __forceinline__ void affine_update(const UpdCtx& u, int n, int j, const float* daff_grad, float* affine,
                                              float* m_aff, float* v_aff) {
  const float beta1w = 0.1f, beta2 = 0.999f, one_m_b2 = 0.001f, eps = 1e-8f;
  const int opt = u.opt;
  const float step_aff = u.step_aff, bc2s = u.bc2s;
  // all four reads before the first store (a read after a store to a possibly aliasing pointer is one more round
  // trip)
  const float g = daff_grad[n * 2 + j];
  const float a = affine[n * 2 + j];
  float m = opt != 1 ? m_aff[n * 2 + j] : 0.0f;
  float vv = opt == 0 ? v_aff[n * 2 + j] : 0.0f;
  if (opt == 0) {
    m = m + beta1w * (g - m);
    vv = vv * beta2;
    vv = vv + one_m_b2 * g * g;
    m_aff[n * 2 + j] = m;
    v_aff[n * 2 + j] = vv;
    float den = sqrtf(vv);
    den = den / bc2s;
    den = den + eps;
    affine[n * 2 + j] = a + (-step_aff) * (m / den);
  } else if (opt == 1) {
    affine[n * 2 + j] = a + (-step_aff) * g;
  } else {
    const float sum = m + g * g;
    m_aff[n * 2 + j] = sum;
    affine[n * 2 + j] = a + (-step_aff) * (g / (sqrtf(sum) + 1e-10f));
  }
}

// opt: 0 Adam (bf16 state m_lat / v_lat), 1 SGD (no state), 2 Adagrad (bf16 state sum in m_lat); the
// affine scalars take the same rule in fp32.  tab per step: Adam [lr_lat/bc1, sqrt(bc2), lr_aff/bc1, 0],
// SGD / Adagrad [lr_lat, 0, lr_aff, 0].
__global__ void latent_update_kernel(bf16* x8, const bf16* v, const bf16* gdir, const bf16* gunet, int hw,
                                     const float* coef, const float* adam_tab, const int* step,
                                     const float* eps_norm, bf16* m_lat, bf16* v_lat, float* affine,
                                     float* m_aff, float* v_aff, const float* daff_grad, float* dbg, int opt,
                                     int kld_mode, float kld_weight) {
  __shared__ float scratch[16];
  const int n = blockIdx.x;
  const int st = *step;
  const float sa = coef[st * 4 + 0], sb = coef[st * 4 + 1], sap = coef[st * 4 + 2], sbp = coef[st * 4 + 3];
  const float step_size = adam_tab[st * 4 + 0], bc2s = adam_tab[st * 4 + 1], step_aff = adam_tab[st * 4 + 2];
  Kld kl{kld_mode, kld_weight, 0.0f, 1.0f, 1.0f / (4.0f * hw)};
  if (kld_mode == 2) {  // mean / biased variance of the latent (bf16 reductions)
    float s1 = 0.0f;
    for (int i = threadIdx.x; i < hw * 4; i += blockDim.x) s1 += (float)x8[((long)n * hw + (i >> 2)) * 8 + 4 + (i & 3)];
    kl.mu = (float)(bf16)(block_sum(s1, scratch) * kl.inv_m);
    __syncthreads();
    float s2 = 0.0f;
    for (int i = threadIdx.x; i < hw * 4; i += blockDim.x) {
      const float d = (float)x8[((long)n * hw + (i >> 2)) * 8 + 4 + (i & 3)] - kl.mu;
      s2 += d * d;
    }
    const float var = (float)(bf16)(block_sum(s2, scratch) * kl.inv_m);
    kl.var_eps = (float)(bf16)(var + 0.0078125f);
    __syncthreads();
  }
  auto grad_at = [&](long pix, int k) {
    float g = (float)(bf16)((float)gdir[pix * 8 + k] + (float)gunet[pix * 8 + k]);
    if (kld_mode) g = (float)(bf16)(g + kl.grad((float)x8[pix * 8 + 4 + k]));
    return g;
  };
  // pass 1: ||g||
  float ss = 0.0f;
  for (int i = threadIdx.x; i < hw * 4; i += blockDim.x) {
    const long pix = (long)n * hw + (i >> 2);
    const int k = i & 3;
    const float g = grad_at(pix, k);
    ss += g * g;
  }
  const float gn = (float)(bf16)sqrtf(block_sum(ss, scratch));
  const float en = eps_norm[n];
  const float gnc = gn < 1e-7f ? (float)(bf16)1e-7f : gn;
  const float factor = (float)(bf16)(en / gnc);
  // pass 2: rescale, Adam (bf16 state), DDIM update with the pre-update v
  const UpdCtx u{sa, sb, sap, sbp, step_size, bc2s, step_aff, opt};
  for (int i = threadIdx.x; i < hw * 4; i += blockDim.x) {
    const long pix = (long)n * hw + (i >> 2);
    const int k = i & 3;
    latent_elem_update(u, x8, v, m_lat, v_lat, pix, k, (float)(bf16)(grad_at(pix, k) * factor));
  }
  if (threadIdx.x < 2) affine_update(u, n, threadIdx.x, daff_grad, affine, m_aff, v_aff);
  if (dbg && threadIdx.x == 0) {
    dbg[n * 4 + 0] = gn;
    dbg[n * 4 + 1] = factor;
  }
}

// Split form of latent_update_kernel (kld_mode 0 / 1, the common case): the single-block update was
// latency-bound at 64 us per step (27 648 scattered 2-B loads per frame through one CU).  Pass 1 gives
// per-block partial sums of g^2, one pixel (4 channels, 8-B loads) per thread; pass 2 folds the frame's
// partials in a fixed order (lane-strided sums + a fixed shuffle tree: deterministic) and applies the
// update to its own pixels.
__global__ void latent_norm_kernel(const bf16* x8, const bf16* gdir, const bf16* gunet, int hw, int kld_mode,
                                   float kld_weight, float* part) {
  __shared__ float scratch[16];
  const int n = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const Kld kl{kld_mode, kld_weight, 0.0f, 1.0f, 1.0f / (4.0f * hw)};
  float ss = 0.0f;
  // the pixel's rows as 16-B loads, unconditional (clamped pixel; skipped below): lane-guarded 2-B loads were one
  // wait each
  const long pix = (long)n * hw + min(p, hw - 1);
  const bf16x8 gd = *reinterpret_cast<const bf16x8*>(gdir + pix * 8);
  const bf16x8 gu = *reinterpret_cast<const bf16x8*>(gunet + pix * 8);
  const bf16x8 xr = *reinterpret_cast<const bf16x8*>(x8 + pix * 8);
  if (p < hw) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float g = (float)(bf16)((float)gd[k] + (float)gu[k]);
      if (kld_mode) g = (float)(bf16)(g + kl.grad((float)xr[4 + k]));
      ss += g * g;
    }
  }
  const float t = block_sum(ss, scratch);
  if (threadIdx.x == 0) part[(long)n * gridDim.x + blockIdx.x] = t;
}

__global__ void latent_apply_kernel(bf16* x8, const bf16* v, const bf16* gdir, const bf16* gunet, int hw,
                                    const float* coef, const float* adam_tab, const int* step, const float* eps_norm,
                                    bf16* m_lat, bf16* v_lat, float* affine, float* m_aff, float* v_aff,
                                    const float* daff_grad, float* dbg, int opt, int kld_mode, float kld_weight,
                                    const float* part) {
  __shared__ float s_ss;
  const int n = blockIdx.y, nblk = gridDim.x;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  // every read of the pixel first (16-B rows, 8-B optimiser state; clamped pixel, skipped below), ahead of the
  // partials' fold and the step's coefficient reads: read per element between the element stores they were ~8
  // dependent round trips
  const long pix = (long)n * hw + min(p, hw - 1);
  const bf16x8 gd = *reinterpret_cast<const bf16x8*>(gdir + pix * 8);
  const bf16x8 gu = *reinterpret_cast<const bf16x8*>(gunet + pix * 8);
  const bf16x8 xr = *reinterpret_cast<const bf16x8*>(x8 + pix * 8);
  const bf16x8 vr = *reinterpret_cast<const bf16x8*>(v + pix * 8);
  const bf16x4 mr = *reinterpret_cast<const bf16x4*>(m_lat + pix * 4);
  const bf16x4 wr = *reinterpret_cast<const bf16x4*>(v_lat + pix * 4);
  if (threadIdx.x < 64) {
    float t = 0.0f;
    for (int b = threadIdx.x; b < nblk; b += 64) t += part[(long)n * nblk + b];
    t = wave_sum(t);
    if (threadIdx.x == 0) s_ss = t;
  }
  __syncthreads();
  const int st = *step;
  const UpdCtx u{coef[st * 4 + 0], coef[st * 4 + 1], coef[st * 4 + 2], coef[st * 4 + 3], adam_tab[st * 4 + 0],
                 adam_tab[st * 4 + 1], adam_tab[st * 4 + 2], opt};
  const float gn = (float)(bf16)sqrtf(s_ss);
  const float en = eps_norm[n];
  const float gnc = gn < 1e-7f ? (float)(bf16)1e-7f : gn;
  const float factor = (float)(bf16)(en / gnc);
  const Kld kl{kld_mode, kld_weight, 0.0f, 1.0f, 1.0f / (4.0f * hw)};
  if (p < hw) {
    bf16x4 xo, mo, wo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float g = (float)(bf16)((float)gd[k] + (float)gu[k]);
      if (kld_mode) g = (float)(bf16)(g + kl.grad((float)xr[4 + k]));
      float m = (float)mr[k], vv = (float)wr[k];
      xo[k] = (bf16)latent_elem_core(u, (float)xr[4 + k], (float)vr[k], (float)(bf16)(g * factor), m, vv);
      mo[k] = (bf16)m;
      wo[k] = (bf16)vv;
    }
    *reinterpret_cast<bf16x4*>(x8 + pix * 8 + 4) = xo;
    if (opt != 1) *reinterpret_cast<bf16x4*>(m_lat + pix * 4) = mo;
    if (opt == 0) *reinterpret_cast<bf16x4*>(v_lat + pix * 4) = wo;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) affine_update(u, n, threadIdx.x, daff_grad, affine, m_aff, v_aff);
  if (dbg && blockIdx.x == 0 && threadIdx.x == 0) {
    dbg[n * 4 + 0] = gn;
    dbg[n * 4 + 1] = factor;
  }
}

// saturates at the last table row, so replays past the end of a call never index beyond [S]
__global__ void step_advance_kernel(int* step, int nsteps) {
  const int s = *step + 1;
  *step = s < nsteps ? s : nsteps - 1;
}

// initial depth latents (marigold_dc.py:677-704): noise [1][4][hw] (NCHW, repeated over frames),
// optional warm start beta*noise + (1-beta)*prev (prev [nb][4][hw]) -> x8[...,4:8]
// noise [noise_frames][4][hw]: one draw shared by every frame (noise_frames 1, marigold_dc.py:677-684), or
// one per frame (noise_frames == nb: the per-seed draws of an ensemble batch)
__global__ void latent_init_kernel(const bf16* noise, int noise_frames, const bf16* prev, float beta, int nb, int hw,
                                   bf16* x8) {
  const long total = (long)nb * hw * 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int p = (int)(i % hw);
    const int k = (int)((i / hw) % 4);
    const long n = i / ((long)hw * 4);
    const long nf = noise_frames > 1 ? n : 0;
    float v = (float)noise[(nf * 4 + k) * hw + p];
    if (prev) {
      const float a = (float)(bf16)(beta * v);
      const float b = (float)(bf16)((1.0f - beta) * (float)prev[i]);
      v = (float)(bf16)(a + b);
    }
    x8[(n * hw + p) * 8 + 4 + k] = (bf16)v;
  }
}

// final dense depth: [nb][1][H][W] fp32 metres
// mode 0: learned affine s^2 (max_g - min_g) aff + sh^2 min_g (marigold_dc.py:323-331);
// mode 1: closed-form scale * aff + shift (marigold_dc.py:332-336), affine from dc_closed_form_affine
__global__ void final_dense_kernel(const bf16* out, int ldo, int nb, int PH, int PW, int RH, int RW, int H, int W,
                                   const float* params, const float* affine, int mode, float* dense) {
  const long total = (long)nb * H * W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % W);
    const int y = (int)((i / W) % H);
    const int n = (int)(i / ((long)H * W));
    Taps t;
    const float* pr = params + n * 8;
    const float aff = sample_affine(out, ldo, n, PH, PW, RH, RW, H, W, y, x, t, interp_nearest(pr));
    const float s = affine[n * 2], sh = affine[n * 2 + 1];
    float F;
    if (mode == 0) {
      const float B = (s * s) * (pr[5] - pr[4]);
      F = B * aff + (sh * sh) * pr[4];
    } else {
      F = s * aff + sh;
    }
    const float G = fminf(fmaxf(F, 0.0f), 1.0f);
    dense[i] = G * (pr[1] - pr[0]) + pr[0];
  }
}

// Plain DDIM step (train_latents=False, marigold_dc.py:905-909): DDIMScheduler.step(v, t, x).prev_sample
// on bf16 tensors, eta = 0, with torch's per-op bf16 rounding (same sequence as latent_update's).
__global__ void ddim_step_kernel(bf16* x8, const bf16* v, long total, const float* coef, const int* step) {
  const int st = *step;
  const float sa = coef[st * 4 + 0], sb = coef[st * 4 + 1], sap = coef[st * 4 + 2], sbp = coef[st * 4 + 3];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i >> 2;
    const int k = (int)(i & 3);
    const float xp = (float)x8[pix * 8 + 4 + k];
    const float vm = (float)v[pix * 8 + k];
    const float x0 = (float)(bf16)((float)(bf16)(sa * xp) - (float)(bf16)(sb * vm));
    const float ep = (float)(bf16)((float)(bf16)(sa * vm) + (float)(bf16)(sb * xp));
    const float dir = (float)(bf16)(sbp * ep);
    x8[pix * 8 + 4 + k] = (bf16)((float)(bf16)(sap * x0) + dir);
  }
}

// compute_affine_params (marigold_dc.py:53-128) over the sparse pixels only (the mask is zero elsewhere),
// one block per frame, with the reference's dtype placement: the affine map is bf16, so its masked sum,
// mean, centred values, squares and variance are bf16-rounded; guides and the covariance are fp32.
// st8 (optional): [nb][8] = (scale, shift, mean a, mean g, var + eps, count) for the differentiated
// full-image form (dc_dense_loss flag 16, dc_closed_form_adjoint)
__global__ void closed_form_kernel(const bf16* out, int ldo, int PH, int PW, int RH, int RW, int H, int W,
                                   const int* idx, const float* gval, const int* cnt, const float* params,
                                   float* affine, float* st8) {
  __shared__ float scratch[16];
  const int n = blockIdx.x;
  const long HW = (long)H * W;
  const int count = cnt[n];
  const int* ix = idx + n * HW;
  const float* gv = gval + n * HW;
  const int nearest = interp_nearest(params + n * 8);
  auto aff_at = [&](int k) {
    const int p = ix[k];
    Taps t;
    return sample_affine(out, ldo, n, PH, PW, RH, RW, H, W, p / W, p - (p / W) * W, t, nearest);
  };
  float sa = 0.0f, sg = 0.0f;
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    sa += aff_at(k);
    sg += gv[k];
  }
  const float sum_a = (float)(bf16)block_sum(sa, scratch);
  __syncthreads();
  const float sum_g = block_sum(sg, scratch);
  __syncthreads();
  const float ma = (float)(bf16)(sum_a / (float)count);
  const float mg = sum_g / (float)count;
  float sv = 0.0f, sc = 0.0f;
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    const float ac = (float)(bf16)(aff_at(k) - ma);
    sv += (float)(bf16)(ac * ac);
    sc += ac * (gv[k] - mg);
  }
  const float var = (float)(bf16)block_sum(sv, scratch);
  __syncthreads();
  const float cov = block_sum(sc, scratch);
  if (threadIdx.x == 0) {
    const float vpe = (float)(bf16)(var + 1e-7f);
    const float scale = cov / vpe;
    if (affine) {
      affine[n * 2] = scale;
      affine[n * 2 + 1] = mg - scale * ma;
    }
    if (st8) {
      float* o = st8 + n * 8;
      o[0] = scale;
      o[1] = mg - scale * ma;
      o[2] = ma;
      o[3] = mg;
      o[4] = vpe;
      o[5] = (float)count;
      o[6] = 0.0f;
      o[7] = 0.0f;
    }
  }
}

// The fit's share of dL/da_k for the full-image closed-form loss: dc_dense_loss (flag 16) leaves
// grad2[n] = (Gs, E) = (sum_p dF_p (a_p - mean a), sum_p dF_p) over every pixel, whose direct term
// s dF_p it has already scattered; the sparse pixels k add Gs (gc_k - 2 s ac_k) / (V + eps) - s E / K
// (the same expression as sparse_loss_cf_kernel's), scattered through the resize taps.  One block per
// frame.
__global__ void cf_adjoint_kernel(const bf16* out, int ldo, int PH, int PW, int RH, int RW, int H, int W,
                                  const int* idx, const float* gval, const int* cnt, const float* params,
                                  const float* st8, const float* grad2, float* dA) {
  const int n = blockIdx.x;
  const long HW = (long)H * W;
  const int count = cnt[n];
  const int* ix = idx + n * HW;
  const float* gv = gval + n * HW;
  const int nearest = interp_nearest(params + n * 8);
  const float* c = st8 + n * 8;
  const float scale = c[0], ma = c[2], mg = c[3], vpe = c[4], K = c[5];
  const float Gs = grad2[n * 2], E = grad2[n * 2 + 1];
  float* dAn = dA + (long)n * PH * PW;
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    const int p = ix[k];
    Taps t;
    const float a = sample_affine(out, ldo, n, PH, PW, RH, RW, H, W, p / W, p - (p / W) * W, t, nearest);
    const float ac = (float)(bf16)(a - ma);
    const float gc = gv[k] - mg;
    const float dff = (float)(bf16)(Gs * (gc - 2.0f * scale * ac) / vpe - scale * E / K);
    if (t.ly1 == 0.0f && t.lx1 == 0.0f && t.y0 == t.y1 && t.x0 == t.x1) {
      atomicAdd(&dAn[(long)t.y0 * PW + t.x0], dff);
    } else {
      atomicAdd(&dAn[(long)t.y0 * PW + t.x0], t.ly0 * t.lx0 * dff);
      atomicAdd(&dAn[(long)t.y0 * PW + t.x1], t.ly0 * t.lx1 * dff);
      atomicAdd(&dAn[(long)t.y1 * PW + t.x0], t.ly1 * t.lx0 * dff);
      atomicAdd(&dAn[(long)t.y1 * PW + t.x1], t.ly1 * t.lx1 * dff);
    }
  }
}

// One optimiser step of the per-input learned affine (train_method="per-input" with full-image losses):
// grad2 [nb][2] from dc_dense_loss, state [nb][4] (Adam m0 v0 m1 v1 / Adagrad sums in m0 m1), `it` the
// 1-based step count; the arithmetic of affine_fit_kernel's step.  One thread per frame.
__global__ void affine_step_kernel(int nb, const float* grad2, int it, float lr, int opt, float* state,
                                   float* affine) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= nb) return;
  const float s = affine[n * 2], sh = affine[n * 2 + 1];
  const float g0 = grad2[n * 2], g1 = grad2[n * 2 + 1];
  float* m = state + n * 4;
  if (opt == 0) {
    double b1p = 1.0, b2p = 1.0;
    for (int i = 0; i < it; ++i) {
      b1p *= 0.9;
      b2p *= 0.999;
    }
    const float step_size = (float)(lr / (1.0 - b1p));
    const float bc2s = (float)sqrt(1.0 - b2p);
    m[0] = m[0] + 0.1f * (g0 - m[0]);
    m[1] = m[1] * 0.999f + 0.001f * g0 * g0;
    m[2] = m[2] + 0.1f * (g1 - m[2]);
    m[3] = m[3] * 0.999f + 0.001f * g1 * g1;
    affine[n * 2] = s + (-step_size) * (m[0] / (sqrtf(m[1]) / bc2s + 1e-8f));
    affine[n * 2 + 1] = sh + (-step_size) * (m[2] / (sqrtf(m[3]) / bc2s + 1e-8f));
  } else if (opt == 1) {
    affine[n * 2] = s + (-lr) * g0;
    affine[n * 2 + 1] = sh + (-lr) * g1;
  } else {
    m[0] = m[0] + g0 * g0;
    m[2] = m[2] + g1 * g1;
    affine[n * 2] = s + (-lr) * (g0 / (sqrtf(m[0]) + 1e-10f));
    affine[n * 2 + 1] = sh + (-lr) * (g1 / (sqrtf(m[2]) + 1e-10f));
  }
}

// Guided steps with closed_form=True (marigold_dc.py:332-336 inside the per-step loop :828-877): the
// affine fit s, t = compute_affine_params(A) of the current preview is differentiated too.  Forward as
// closed_form_kernel; with e_k = dL/dd_k (l1 + l2, clamp(0, 1) mask), Gs = sum e_k (a_k - mean a),
// E = sum e_k, V the masked variance, centred a / g written ac_k / gc_k:
//   dL/da_k = s e_k + Gs (gc_k - 2 s ac_k) / (V + eps) - s E / K
// scattered through the bilinear taps into dA like sparse_loss_kernel.  One block per frame.
__global__ void sparse_loss_cf_kernel(const bf16* out, int ldo, int PH, int PW, int RH, int RW, int H, int W,
                                      const int* idx, const float* gval, const int* cnt, const float* params,
                                      float* dA, float* loss) {
  __shared__ float scratch[16];
  const int n = blockIdx.x;
  const long HW = (long)H * W;
  const int count = cnt[n];
  const int* ix = idx + n * HW;
  const float* gv = gval + n * HW;
  const int nearest = interp_nearest(params + n * 8);
  auto aff_at = [&](int k, Taps& t) {
    const int p = ix[k];
    return sample_affine(out, ldo, n, PH, PW, RH, RW, H, W, p / W, p - (p / W) * W, t, nearest);
  };
  float sa = 0.0f, sg = 0.0f;
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    Taps t;
    sa += aff_at(k, t);
    sg += gv[k];
  }
  const float sum_a = (float)(bf16)block_sum(sa, scratch);
  __syncthreads();
  const float sum_g = block_sum(sg, scratch);
  __syncthreads();
  const float K = (float)count;
  const float ma = (float)(bf16)(sum_a / K);
  const float mg = sum_g / K;
  float sv = 0.0f, sc = 0.0f;
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    Taps t;
    const float ac = (float)(bf16)(aff_at(k, t) - ma);
    sv += (float)(bf16)(ac * ac);
    sc += ac * (gv[k] - mg);
  }
  const float var = (float)(bf16)block_sum(sv, scratch);
  __syncthreads();
  const float cov = block_sum(sc, scratch);
  __syncthreads();
  const float vpe = (float)(bf16)(var + 1e-7f);
  const float scale = cov / vpe;
  const float shift = mg - scale * ma;
  const float inv_cnt = 1.0f / K;
  const DSpace ds(params + n * 8);
  float se = 0.0f, sge = 0.0f, lsum = 0.0f;
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    Taps t;
    const float a = aff_at(k, t);
    const float F = scale * a + shift;
    float dNdG;
    const float Nv = ds(fminf(fmaxf(F, 0.0f), 1.0f), dNdG);
    const float r = Nv - gv[k];
    lsum += fabsf(r) * inv_cnt + (r * r) * inv_cnt;
    const float sgn = (r > 0.0f) ? 1.0f : ((r < 0.0f) ? -1.0f : 0.0f);
    const float dF = (F >= 0.0f && F <= 1.0f) ? (sgn * inv_cnt + 2.0f * r * inv_cnt) * dNdG : 0.0f;
    se += dF;
    sge += dF * (a - ma);
  }
  const float E = block_sum(se, scratch);
  __syncthreads();
  const float Gs = block_sum(sge, scratch);
  __syncthreads();
  const float ls = block_sum(lsum, scratch);
  float* dAn = dA + (long)n * PH * PW;
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    Taps t;
    const float a = aff_at(k, t);
    const float F = scale * a + shift;
    float dNdG;
    const float Nv = ds(fminf(fmaxf(F, 0.0f), 1.0f), dNdG);
    const float r = Nv - gv[k];
    const float sgn = (r > 0.0f) ? 1.0f : ((r < 0.0f) ? -1.0f : 0.0f);
    const float e = (F >= 0.0f && F <= 1.0f) ? (sgn * inv_cnt + 2.0f * r * inv_cnt) * dNdG : 0.0f;
    const float ac = (float)(bf16)(a - ma);
    const float gc = gv[k] - mg;
    const float dff = (float)(bf16)(scale * e + Gs * (gc - 2.0f * scale * ac) / vpe - scale * E * inv_cnt);
    if (t.ly1 == 0.0f && t.lx1 == 0.0f && t.y0 == t.y1 && t.x0 == t.x1) {
      atomicAdd(&dAn[(long)t.y0 * PW + t.x0], dff);
    } else {
      atomicAdd(&dAn[(long)t.y0 * PW + t.x0], t.ly0 * t.lx0 * dff);
      atomicAdd(&dAn[(long)t.y0 * PW + t.x1], t.ly0 * t.lx1 * dff);
      atomicAdd(&dAn[(long)t.y1 * PW + t.x0], t.ly1 * t.lx0 * dff);
      atomicAdd(&dAn[(long)t.y1 * PW + t.x1], t.ly1 * t.lx1 * dff);
    }
  }
  if (threadIdx.x == 0) loss[n] = ls;
}

// Per-input training (train_method="per-input", marigold_dc.py:911-967) with learned affine params: the
// reference's optimiser still holds the pre-loop latent tensor (:777-783 vs :913), so only scale / shift
// move; the decode A of the final latents is fixed, and each of the train_steps iterations is the l1 + l2
// loss on the UNclamped s^2 (max - min) A + sh^2 min at the sparse pixels followed by one fp32 optimiser
// step (opt 0 Adam with step count 1..train_steps, 1 SGD, 2 Adagrad; torch.optim arithmetic).  One block
// per frame, all steps in one launch.
__global__ void affine_fit_kernel(const bf16* out, int ldo, int PH, int PW, int RH, int RW, int H, int W,
                                  const int* idx, const float* gval, const int* cnt, const float* params,
                                  int train_steps, float lr, int opt, float* affine, float* loss) {
  __shared__ float scratch[16];
  __shared__ float s_aff[2];
  const int n = blockIdx.x;
  const long HW = (long)H * W;
  const int count = cnt[n];
  const int* ix = idx + n * HW;
  const float* gv = gval + n * HW;
  const float* pr = params + n * 8;
  const float gmin = pr[4], gmax = pr[5];
  const float inv_cnt = 1.0f / (float)count;
  const DSpace ds(pr);
  const float beta1w = 0.1f, beta2 = 0.999f, one_m_b2 = 0.001f, eps = 1e-8f;
  float m0 = 0.0f, v0 = 0.0f, m1 = 0.0f, v1 = 0.0f;
  if (threadIdx.x == 0) {
    s_aff[0] = affine[n * 2];
    s_aff[1] = affine[n * 2 + 1];
  }
  __syncthreads();
  double b1p = 1.0, b2p = 1.0;
  for (int it = 1; it <= train_steps; ++it) {
    const float s = s_aff[0], sh = s_aff[1];
    const float B = (s * s) * (gmax - gmin);
    const float E = (sh * sh) * gmin;
    float sum_db = 0.0f, sum_de = 0.0f, lsum = 0.0f;
    for (int k = threadIdx.x; k < count; k += blockDim.x) {
      const int p = ix[k];
      Taps t;
      const float a = sample_affine(out, ldo, n, PH, PW, RH, RW, H, W, p / W, p - (p / W) * W, t, interp_nearest(pr));
      const float F = B * a + E;
      float dNdF;
      const float Nv = ds(F, dNdF);
      const float r = Nv - gv[k];
      lsum += fabsf(r) * inv_cnt + (r * r) * inv_cnt;
      const float sgn = (r > 0.0f) ? 1.0f : ((r < 0.0f) ? -1.0f : 0.0f);
      const float dF = (sgn * inv_cnt + 2.0f * r * inv_cnt) * dNdF;
      sum_db += dF * a;
      sum_de += dF;
    }
    const float db = block_sum(sum_db, scratch);
    __syncthreads();
    const float de = block_sum(sum_de, scratch);
    __syncthreads();
    const float ls = block_sum(lsum, scratch);
    __syncthreads();
    if (threadIdx.x == 0) {
      b1p *= 0.9;
      b2p *= 0.999;
      const float step_size = (float)(lr / (1.0 - b1p));
      const float bc2s = (float)sqrt(1.0 - b2p);
      const float g0 = db * (gmax - gmin) * (2.0f * s), g1 = (de * gmin) * (2.0f * sh);
      if (opt == 0) {
        m0 = m0 + beta1w * (g0 - m0);
        v0 = v0 * beta2 + one_m_b2 * g0 * g0;
        m1 = m1 + beta1w * (g1 - m1);
        v1 = v1 * beta2 + one_m_b2 * g1 * g1;
        s_aff[0] = s + (-step_size) * (m0 / (sqrtf(v0) / bc2s + eps));
        s_aff[1] = sh + (-step_size) * (m1 / (sqrtf(v1) / bc2s + eps));
      } else if (opt == 1) {
        s_aff[0] = s + (-lr) * g0;
        s_aff[1] = sh + (-lr) * g1;
      } else {  // Adagrad: m0 / m1 hold the squared-gradient sums
        m0 = m0 + g0 * g0;
        m1 = m1 + g1 * g1;
        s_aff[0] = s + (-lr) * (g0 / (sqrtf(m0) + 1e-10f));
        s_aff[1] = sh + (-lr) * (g1 / (sqrtf(m1) + 1e-10f));
      }
      loss[n] = ls;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    affine[n * 2] = s_aff[0];
    affine[n * 2 + 1] = s_aff[1];
  }
}

// ---------------------------------------------------------------- full-image losses
// compute_loss with edge / smooth terms (marigold_dc.py:195-235) needs the whole dense map, not only the
// sparse pixels.  Three launches per guided step (only when loss_funcs is not {l1, l2}):
//   dense_map    N (the clamped, learned-affine depth in the loss's depth space) at every (y, x)
//   dense_grad   per pixel: dL/dN from the l1 / l2 term (sparse pixels, guide map) and from the four
//                neighbour pairs of the edge / smooth terms (gathered, no atomics), chained through the
//                depth space, clamp and affine into dA (resize adjoint) and per-block sums of the loss,
//                dL/d(s^2 (max-min)) and dL/d(sh^2 min) in a fixed order
//   dense_fold   one block per frame folds the block sums in order -> loss, d scale, d shift
// flags: 1 l1, 2 l2, 4 edge, 8 smooth; 16 closed-form affine (affine = dc_closed_form_stats' [nb][8],
// d = scale a + shift; the fold leaves (Gs, E) for dc_closed_form_adjoint), 32 no clamp(0, 1) (per-input
// training, marigold_dc.py:928-929), 64 no dA (affine-only gradient).  gray = 0.299 R + 0.587 G +
// 0.114 B of the uint8 image, in fp32 as torch forms it (uint8 * python float -> float32).
struct DenseCtx {
  const bf16* out;
  int ldo, PH, PW, RH, RW, H, W;
  const float* params;
  const float* affine;
  int cf, noclamp;
};

// returns N; aff = the resized decode, F = the affine value, B = dF/daff
__device__ __forceinline__ float dense_value(const DenseCtx& c, int n, int y, int x, float& aff, float& F, float& dNdG,
                                             Taps& t, float& B) {
  const float* pr = c.params + n * 8;
  aff = sample_affine(c.out, c.ldo, n, c.PH, c.PW, c.RH, c.RW, c.H, c.W, y, x, t, interp_nearest(pr));
  if (c.cf) {
    B = c.affine[n * 8];
    F = B * aff + c.affine[n * 8 + 1];
  } else {
    const float s = c.affine[n * 2], sh = c.affine[n * 2 + 1];
    B = (s * s) * (pr[5] - pr[4]);
    F = B * aff + (sh * sh) * pr[4];
  }
  const DSpace ds(pr);
  return ds(c.noclamp ? F : fminf(fmaxf(F, 0.0f), 1.0f), dNdG);
}

__device__ __forceinline__ float gray_at(const unsigned char* img, int n, long HW, long p) {
  const unsigned char* b = img + (long)n * 3 * HW + p;
  return (0.299f * (float)b[0] + 0.587f * (float)b[HW]) + 0.114f * (float)b[2 * HW];
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }

__global__ void dense_map_kernel(DenseCtx c, float* nmap) {
  const int n = blockIdx.y;
  const long HW = (long)c.H * c.W;
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HW) return;
  float aff, F, dNdG, B;
  Taps t;
  nmap[n * HW + p] = dense_value(c, n, (int)(p / c.W), (int)(p % c.W), aff, F, dNdG, t, B);
}

// part[n][block][3] = (loss, sum dF * aff, sum dF)
__global__ void dense_grad_kernel(DenseCtx c, const unsigned char* img, const float* nmap, const float* gmap,
                                  const int* cnt, int flags, float* dA, float* part) {  // dA null: no scatter
  __shared__ float scratch[16];
  const int n = blockIdx.y;
  const int H = c.H, W = c.W;
  const long HW = (long)H * W;
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float lsum = 0.0f, sdb = 0.0f, sde = 0.0f;
  if (p < HW) {
    const int y = (int)(p / W), x = (int)(p % W);
    float aff, F, dNdG, B;
    Taps t;
    const float Nv = dense_value(c, n, y, x, aff, F, dNdG, t, B);
    const float* nm = nmap + n * HW;
    float gN = 0.0f;
    // l1 / l2 at the sparse pixels (guide map holds NaN elsewhere)
    const float gv = gmap[n * HW + p];
    if ((flags & 3) && !__builtin_isnan(gv)) {
      const float inv_cnt = 1.0f / (float)cnt[n];
      const float r = Nv - gv;
      if (flags & 1) { lsum += fabsf(r) * inv_cnt; gN += sgnf(r) * inv_cnt; }
      if (flags & 2) { lsum += (r * r) * inv_cnt; gN += 2.0f * r * inv_cnt; }
    }
    if (flags & 12) {
      const float icx = 1.0f / (float)((long)H * (W - 1)), icy = 1.0f / (float)((long)(H - 1) * W);
      const bool edge = flags & 4, smooth = flags & 8;
      float gp = 0.0f;
      if (edge) gp = gray_at(img, n, HW, p);
      // pair (p, right): owned by p (loss), contributes +c to p; pair (left, p): -c to p
      auto pair = [&](float a, float b, float ga, float gb, float ic, bool own) {
        const float d = a - b;
        float cval = 0.0f;
        if (edge) {
          const float g = fabsf(ga - gb);
          const float e = fabsf(d) - g;
          if (own) lsum += fabsf(e) * ic;
          cval += sgnf(e) * ic * sgnf(d);
        }
        if (smooth) {
          if (own) lsum += fabsf(d) * ic;
          cval += ic * sgnf(d);
        }
        return cval;
      };
      if (x + 1 < W) gN += pair(Nv, nm[p + 1], gp, edge ? gray_at(img, n, HW, p + 1) : 0.0f, icx, true);
      if (x > 0) gN -= pair(nm[p - 1], Nv, edge ? gray_at(img, n, HW, p - 1) : 0.0f, gp, icx, false);
      if (y + 1 < H) gN += pair(Nv, nm[p + W], gp, edge ? gray_at(img, n, HW, p + W) : 0.0f, icy, true);
      if (y > 0) gN -= pair(nm[p - W], Nv, edge ? gray_at(img, n, HW, p - W) : 0.0f, gp, icy, false);
    }
    const float dF = (c.noclamp || (F >= 0.0f && F <= 1.0f)) ? gN * dNdG : 0.0f;
    sdb = dF * aff;
    sde = dF;
    if (dF != 0.0f && dA) {
      const float dff = (float)(bf16)(dF * B);
      float* dAn = dA + (long)n * c.PH * c.PW;
      if (t.ly1 == 0.0f && t.lx1 == 0.0f && t.y0 == t.y1 && t.x0 == t.x1) {
        atomicAdd(&dAn[(long)t.y0 * c.PW + t.x0], dff);
      } else {
        atomicAdd(&dAn[(long)t.y0 * c.PW + t.x0], t.ly0 * t.lx0 * dff);
        atomicAdd(&dAn[(long)t.y0 * c.PW + t.x1], t.ly0 * t.lx1 * dff);
        atomicAdd(&dAn[(long)t.y1 * c.PW + t.x0], t.ly1 * t.lx0 * dff);
        atomicAdd(&dAn[(long)t.y1 * c.PW + t.x1], t.ly1 * t.lx1 * dff);
      }
    }
  }
  const float l = block_sum(lsum, scratch);
  __syncthreads();
  const float db = block_sum(sdb, scratch);
  __syncthreads();
  const float de = block_sum(sde, scratch);
  if (threadIdx.x == 0) {
    float* o = part + ((long)n * gridDim.x + blockIdx.x) * 3;
    o[0] = l;
    o[1] = db;
    o[2] = de;
  }
}

__global__ void dense_fold_kernel(const float* part, int nblk, const float* params, const float* affine, int cf,
                                  float* daff_grad, float* loss) {
  __shared__ float scratch[16];
  const int n = blockIdx.x;
  float l = 0.0f, db = 0.0f, de = 0.0f;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
    const float* o = part + ((long)n * nblk + b) * 3;
    l += o[0];
    db += o[1];
    de += o[2];
  }
  l = block_sum(l, scratch);
  __syncthreads();
  db = block_sum(db, scratch);
  __syncthreads();
  de = block_sum(de, scratch);
  if (threadIdx.x == 0) {
    if (cf) {   // (Gs, E) for cf_adjoint_kernel
      daff_grad[n * 2] = db - affine[n * 8 + 2] * de;
      daff_grad[n * 2 + 1] = de;
    } else {
      const float* pr = params + n * 8;
      const float s = affine[n * 2], sh = affine[n * 2 + 1];
      daff_grad[n * 2] = (db * (pr[5] - pr[4])) * (2.0f * s);
      daff_grad[n * 2 + 1] = (de * pr[4]) * (2.0f * sh);
    }
    loss[n] = l;
  }
}

// dense guide map [nb][H*W]: the normalised guide at the sparse pixels, NaN elsewhere
__global__ void guide_map_kernel(const int* idx, const float* gval, const int* cnt, long HW, float* gmap) {
  const int n = blockIdx.y;
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += (long)gridDim.x * blockDim.x)
    gmap[n * HW + p] = __int_as_float(0x7fc00000);
}
__global__ void guide_scatter_kernel(const int* idx, const float* gval, const int* cnt, long HW, float* gmap) {
  const int n = blockIdx.y;
  for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < cnt[n]; k += (long)gridDim.x * blockDim.x)
    gmap[n * HW + idx[n * HW + k]] = gval[n * HW + k];
}

inline dim3 grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 65536) b = 65536;
  return dim3((unsigned)(b < 1 ? 1 : b));
}

}  // namespace

extern "C" int dc_sparse_setup(const float* sparse, int nb, int h, int w, int norm, float min_depth, float max_depth,
                               const float* host_lohi, int projection, int inv, int interp, int* idx, float* gval,
                               int* cnt, float* params, void* stream) {
  if (!sparse || !idx || !gval || !cnt || !params || nb <= 0 || h <= 0 || w <= 0) return DC_ERR_ARG;
  if (norm < 0 || norm > 2 || projection < 0 || projection > 2 || inv < 0 || inv > 1 || interp < 0 || interp > 1)
    return DC_ERR_ARG;
  if (norm == 2 && !host_lohi) return DC_ERR_ARG;
  hipLaunchKernelGGL(sparse_setup_kernel, dim3(nb), dim3(SETUP_THREADS), 0, (hipStream_t)stream, sparse, h, w, norm,
                     min_depth, max_depth, host_lohi, projection, inv, interp, idx, gval, cnt, params);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_preview(const void* x8, const void* v, int nb, int hw, const float* coef, const int* step, void* x0,
                          void* tin, float* eps_norm, void* stream) {
  if (!x8 || !v || !coef || !step || !x0 || !tin || !eps_norm || nb <= 0 || hw <= 0) return DC_ERR_ARG;
  hipLaunchKernelGGL(preview_kernel, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (const bf16*)x8, (const bf16*)v, hw,
                     coef, step, (bf16*)x0, (bf16*)tin, eps_norm);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_sparse_loss(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                              const int* idx, const float* gval, const int* cnt, const float* params,
                              const float* affine, float* dA, float* daff_grad, float* loss, void* stream) {
  if (!dec_out || !idx || !gval || !cnt || !params || !affine || !dA || !daff_grad || !loss) return DC_ERR_ARG;
  if (nb <= 0 || rh > ph || rw > pw || h <= 0 || w <= 0) return DC_ERR_ARG;
  hipLaunchKernelGGL(sparse_loss_kernel, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (const bf16*)dec_out, ldo, ph,
                     pw, rh, rw, h, w, idx, gval, cnt, params, affine, dA, daff_grad, loss);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_decode_tail_bwd(const void* dec_out, int ldo, const float* dA, int nb, int ph, int pw, int rh,
                                  int rw, void* dout, void* stream) {
  if (!dec_out || !dA || !dout || nb <= 0) return DC_ERR_ARG;
  hipLaunchKernelGGL(decode_tail_bwd_kernel, grid_for((long)nb * ph * pw), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)dec_out, ldo, dA, nb, ph, pw, rh, rw, (bf16*)dout);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_latent_update(void* x8, const void* v, const void* gdir, const void* gunet, int nb, int hw,
                                const float* coef, const float* adam_tab, const int* step, const float* eps_norm,
                                void* m_lat, void* v_lat, float* affine, float* m_aff, float* v_aff,
                                const float* daff_grad, float* dbg, int opt, int kld_mode, float kld_weight,
                                float* ws, long long ws_bytes, void* stream) {
  if (!x8 || !v || !gdir || !gunet || !coef || !adam_tab || !step || !eps_norm || !m_lat || !v_lat || !affine ||
      !m_aff || !v_aff || !daff_grad || nb <= 0 || hw <= 0 || opt < 0 || opt > 2 || kld_mode < 0 || kld_mode > 2)
    return DC_ERR_ARG;
  const int nblk = (hw + 255) / 256;
  const char* split_env = getenv("DC_LU_SPLIT");   // 0: the single-block form (A/B)
  if (ws && kld_mode != 2 && (long long)nb * nblk * 4 <= ws_bytes && !(split_env && atoi(split_env) == 0)) {
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(latent_norm_kernel, dim3(nblk, nb), dim3(256), 0, st, (const bf16*)x8, (const bf16*)gdir,
                       (const bf16*)gunet, hw, kld_mode, kld_weight, ws);
    hipLaunchKernelGGL(latent_apply_kernel, dim3(nblk, nb), dim3(256), 0, st, (bf16*)x8, (const bf16*)v,
                       (const bf16*)gdir, (const bf16*)gunet, hw, coef, adam_tab, step, eps_norm, (bf16*)m_lat,
                       (bf16*)v_lat, affine, m_aff, v_aff, daff_grad, dbg, opt, kld_mode, kld_weight, ws);
    DC_CHECK_LAUNCH();
    return DC_OK;
  }
  hipLaunchKernelGGL(latent_update_kernel, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (bf16*)x8, (const bf16*)v,
                     (const bf16*)gdir, (const bf16*)gunet, hw, coef, adam_tab, step, eps_norm, (bf16*)m_lat,
                     (bf16*)v_lat, affine, m_aff, v_aff, daff_grad, dbg, opt, kld_mode, kld_weight);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_step_advance(int* step, int nsteps, void* stream) {
  if (!step || nsteps <= 0) return DC_ERR_ARG;
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step, nsteps);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_latent_init(const void* noise, int noise_frames, const void* prev, float beta, int nb, int hw,
                              void* x8, void* stream) {
  if (!noise || !x8 || nb <= 0 || hw <= 0 || (noise_frames != 1 && noise_frames != nb)) return DC_ERR_ARG;
  hipLaunchKernelGGL(latent_init_kernel, grid_for((long)nb * hw * 4), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)noise, noise_frames, (const bf16*)prev, beta, nb, hw, (bf16*)x8);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_final_dense(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                              const float* params, const float* affine, int mode, float* dense, void* stream) {
  if (!dec_out || !params || !affine || !dense || nb <= 0 || mode < 0 || mode > 1) return DC_ERR_ARG;
  hipLaunchKernelGGL(final_dense_kernel, grid_for((long)nb * h * w), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)dec_out, ldo, nb, ph, pw, rh, rw, h, w, params, affine, mode, dense);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_ddim_step(void* x8, const void* v, int nb, int hw, const float* coef, const int* step,
                            void* stream) {
  if (!x8 || !v || !coef || !step || nb <= 0 || hw <= 0) return DC_ERR_ARG;
  const long total = (long)nb * hw * 4;
  hipLaunchKernelGGL(ddim_step_kernel, grid_for(total), dim3(256), 0, (hipStream_t)stream, (bf16*)x8,
                     (const bf16*)v, total, coef, step);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_closed_form_affine(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h,
                                     int w, const int* idx, const float* gval, const int* cnt, const float* params,
                                     float* affine, void* stream) {
  if (!dec_out || !idx || !gval || !cnt || !params || !affine || nb <= 0) return DC_ERR_ARG;
  hipLaunchKernelGGL(closed_form_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const bf16*)dec_out, ldo, ph,
                     pw, rh, rw, h, w, idx, gval, cnt, params, affine, (float*)nullptr);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_closed_form_stats(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h,
                                    int w, const int* idx, const float* gval, const int* cnt, const float* params,
                                    float* st8, void* stream) {
  if (!dec_out || !idx || !gval || !cnt || !params || !st8 || nb <= 0 || rh > ph || rw > pw) return DC_ERR_ARG;
  hipLaunchKernelGGL(closed_form_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const bf16*)dec_out, ldo, ph,
                     pw, rh, rw, h, w, idx, gval, cnt, params, (float*)nullptr, st8);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_closed_form_adjoint(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h,
                                      int w, const int* idx, const float* gval, const int* cnt, const float* params,
                                      const float* st8, const float* grad2, float* dA, void* stream) {
  if (!dec_out || !idx || !gval || !cnt || !params || !st8 || !grad2 || !dA || nb <= 0 || rh > ph || rw > pw)
    return DC_ERR_ARG;
  hipLaunchKernelGGL(cf_adjoint_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const bf16*)dec_out, ldo, ph,
                     pw, rh, rw, h, w, idx, gval, cnt, params, st8, grad2, dA);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_affine_step(int nb, const float* grad2, int it, float lr, int opt, float* state, float* affine,
                              void* stream) {
  if (nb <= 0 || !grad2 || !state || !affine || it <= 0 || opt < 0 || opt > 2) return DC_ERR_ARG;
  hipLaunchKernelGGL(affine_step_kernel, dim3((nb + 63) / 64), dim3(64), 0, (hipStream_t)stream, nb, grad2, it, lr,
                     opt, state, affine);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// byte fill by a kernel (16-B vector stores, byte-granular head / tail), not hipMemsetAsync: replayed from a
// hipGraph in a later call, the memset node that hipMemsetAsync captures did not clear the guided step's dA
// gradient map (the replay kept the previous call's values, tools/diag_batch.py DIAG=state / sync; with this
// kernel every replay equals the eager step bitwise), so every fill of the library is a kernel node
__global__ void fill_bytes_kernel(unsigned char* p, unsigned char v, long long head, long long nvec, long long bytes) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned w = 0x01010101u * v;
  const uint4 q = make_uint4(w, w, w, w);
  uint4* pv = reinterpret_cast<uint4*>(p + head);
  for (long long i = t0; i < nvec; i += stride) pv[i] = q;
  for (long long i = t0; i < head; i += stride) p[i] = v;
  for (long long i = head + nvec * 16 + t0; i < bytes; i += stride) p[i] = v;
}

extern "C" int dc_memset_async(void* ptr, int value, long long bytes, void* stream) {
  if (!ptr || bytes < 0) return DC_ERR_ARG;
  if (bytes == 0) return DC_OK;
  unsigned char* p = (unsigned char*)ptr;
  long long head = (16 - ((uintptr_t)p & 15)) & 15;
  if (head > bytes) head = bytes;
  const long long nvec = (bytes - head) / 16;
  const long long blocks = std::min<long long>(4096, std::max<long long>(1, (nvec + 255) / 256));
  hipLaunchKernelGGL(fill_bytes_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p,
                     (unsigned char)value, head, nvec, bytes);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_sparse_loss_cf(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                                 const int* idx, const float* gval, const int* cnt, const float* params, float* dA,
                                 float* loss, void* stream) {
  if (!dec_out || !idx || !gval || !cnt || !params || !dA || !loss || nb <= 0 || rh > ph || rw > pw)
    return DC_ERR_ARG;
  hipLaunchKernelGGL(sparse_loss_cf_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const bf16*)dec_out, ldo,
                     ph, pw, rh, rw, h, w, idx, gval, cnt, params, dA, loss);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_affine_fit(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                             const int* idx, const float* gval, const int* cnt, const float* params, int train_steps,
                             float lr, int opt, float* affine, float* loss, void* stream) {
  if (!dec_out || !idx || !gval || !cnt || !params || !affine || !loss || nb <= 0 || train_steps <= 0 ||
      rh > ph || rw > pw || opt < 0 || opt > 2)
    return DC_ERR_ARG;
  hipLaunchKernelGGL(affine_fit_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const bf16*)dec_out, ldo, ph,
                     pw, rh, rw, h, w, idx, gval, cnt, params, train_steps, lr, opt, affine, loss);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" long long dc_dense_loss_ws_bytes(int nb, int h, int w) {
  if (nb <= 0 || h <= 0 || w <= 0) return -1;
  const long HW = (long)h * w;
  const long nblk = (HW + 255) / 256;
  return (long long)(nb * HW + nb * nblk * 3) * (long long)sizeof(float);
}

extern "C" int dc_guide_map(const int* idx, const float* gval, const int* cnt, int nb, int h, int w, float* gmap,
                            void* stream) {
  if (!idx || !gval || !cnt || !gmap || nb <= 0 || h <= 0 || w <= 0) return DC_ERR_ARG;
  const long HW = (long)h * w;
  const dim3 g((unsigned)min((HW + 255) / 256, 4096L), nb);
  hipLaunchKernelGGL(guide_map_kernel, g, dim3(256), 0, (hipStream_t)stream, idx, gval, cnt, HW, gmap);
  hipLaunchKernelGGL(guide_scatter_kernel, g, dim3(256), 0, (hipStream_t)stream, idx, gval, cnt, HW, gmap);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_dense_loss(const void* dec_out, int ldo, int nb, int ph, int pw, int rh, int rw, int h, int w,
                             const unsigned char* imgs, const float* gmap, const int* cnt, const float* params,
                             const float* affine, int flags, float* ws, float* dA, float* daff_grad, float* loss,
                             void* stream) {
  if (!dec_out || !gmap || !cnt || !params || !affine || !ws || !daff_grad || !loss) return DC_ERR_ARG;
  if (nb <= 0 || rh > ph || rw > pw || h < 2 || w < 2 || (flags & 15) == 0 || flags > 127) return DC_ERR_ARG;
  if ((flags & 4) && !imgs) return DC_ERR_ARG;
  if (!(flags & 64) && !dA) return DC_ERR_ARG;
  const DenseCtx c{(const bf16*)dec_out, ldo, ph, pw, rh, rw, h, w, params, affine, (flags >> 4) & 1, (flags >> 5) & 1};
  const int lf = flags & 15;
  if (flags & 64) dA = nullptr;
  const long HW = (long)h * w;
  const int nblk = (int)((HW + 255) / 256);
  float* nmap = ws;
  float* part = ws + (long)nb * HW;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dense_map_kernel, dim3(nblk, nb), dim3(256), 0, st, c, nmap);
  hipLaunchKernelGGL(dense_grad_kernel, dim3(nblk, nb), dim3(256), 0, st, c, imgs, nmap, gmap, cnt, lf, dA, part);
  hipLaunchKernelGGL(dense_fold_kernel, dim3(nb), dim3(256), 0, st, part, nblk, params, affine, c.cf, daff_grad, loss);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

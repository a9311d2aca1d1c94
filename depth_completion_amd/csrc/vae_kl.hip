// Kernels of the AutoencoderKL path (`--vae original`, predict.py:44-52) that the conv / norm kernels do
// not cover (gfx950):
//   * the latent scaling of decode_prediction (vae.decode(z / scaling_factor)) and its backward chained
//     into the Tweedie preview (the TAESD path's tanh clamp is replaced by the division);
//   * the single-head mid-block attention (head dim = 512 channels, too wide for the flash kernels) as
//     GEMMs on dc_conv_gemm around a row softmax: S = Q K^T, P = softmax(S / sqrt(C)), O = P V, and
//     its backward dS = P (dP - rowsum(P dP)) / sqrt(C), with the [T][T] matrices in HBM (T = latent
//     pixels: 6912 at 768 x 576, 95 MB in bf16) and a tiled transpose for the operands the GEMM wants
//     K-contiguous.
// Softmax arithmetic is fp32 on bf16 scores; probabilities and score gradients are stored in bf16.
#include "common.h"
#include "../../include/dcamd.h"

namespace {

inline dim3 grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 65536) b = 65536;
  return dim3((unsigned)(b < 1 ? 1 : b));
}

// y[p][k] = bf16(x[p][k] / s) for the 4 latent channels, 0 for 4..7
__global__ void latent_scale_fwd_kernel(const bf16* x, int ldx, long P, float s, bf16* y) {
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
    float o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = (float)x[p * ldx + k] / s;
      o[k + 4] = 0.0f;
    }
    store8(y + p * 8, o);
  }
}

// backward of z / s (bf16 autograd: g / s rounded), then of x0 = sqrt(a) x - sqrt(1-a) v as in
// taesd_clamp_bwd: gx_direct = g sqrt(a), dv = -g sqrt(1-a)
__global__ void latent_scale_bwd_kernel(const bf16* dy, int lddy, long P, float s, const float* coef,
                                        const int* step, bf16* gx_direct, bf16* dv) {
  const float sa = coef[*step * 4 + 0], sb = coef[*step * 4 + 1];
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
    float gd[8], vv[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float g = (float)(bf16)((float)dy[p * lddy + k] / s);
      gd[k] = g * sa;
      vv[k] = -g * sb;
      gd[k + 4] = 0.0f;
      vv[k + 4] = 0.0f;
    }
    store8(gx_direct + p * 8, gd);
    store8(dv + p * 8, vv);
  }
}

constexpr int kSmThreads = 256;

__device__ float block_max_f(float v, float* sh) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = l < (kSmThreads >> 6) ? sh[l] : -INFINITY;
  return wave_max(t);
}

// one block per row: P[r][c] = exp(S[r][c] * scale - m) / sum, c < cols; P[r][cols .. ldp) = 0
__global__ __launch_bounds__(kSmThreads) void softmax_rows_kernel(const bf16* S, int lds, int cols, float scale,
                                                                  bf16* Pm, int ldp) {
  __shared__ float sh[16];
  const long r = blockIdx.x;
  const bf16* srow = S + r * lds;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < cols; c += kSmThreads) m = fmaxf(m, (float)srow[c] * scale);
  m = block_max_f(m, sh);
  float sum = 0.0f;
  for (int c = threadIdx.x; c < cols; c += kSmThreads) sum += __expf((float)srow[c] * scale - m);
  sum = block_sum(sum, sh);
  const float inv = 1.0f / sum;
  bf16* prow = Pm + r * ldp;
  for (int c = threadIdx.x; c < ldp; c += kSmThreads)
    prow[c] = c < cols ? (bf16)(__expf((float)srow[c] * scale - m) * inv) : (bf16)0.0f;
}

// one block per row: dS = P (dP - sum_c P dP) * scale, zero past cols
__global__ __launch_bounds__(kSmThreads) void softmax_rows_bwd_kernel(const bf16* Pm, int ldp, const bf16* dP,
                                                                      int lddp, int cols, float scale, bf16* dS,
                                                                      int ldds) {
  __shared__ float sh[16];
  const long r = blockIdx.x;
  const bf16* prow = Pm + r * ldp;
  const bf16* drow = dP + r * lddp;
  float dot = 0.0f;
  for (int c = threadIdx.x; c < cols; c += kSmThreads) dot += (float)prow[c] * (float)drow[c];
  dot = block_sum(dot, sh);
  bf16* orow = dS + r * ldds;
  for (int c = threadIdx.x; c < ldds; c += kSmThreads)
    orow[c] = c < cols ? (bf16)((float)prow[c] * ((float)drow[c] - dot) * scale) : (bf16)0.0f;
}

// y[c][r] = x[r][c] (r < rows, c < cols), y[c][rows .. ldy) = 0: 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void transpose_kernel(const bf16* x, int ldx, int rows, int cols, bf16* y,
                                                        int ldy) {
  __shared__ bf16 tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < rows && c < cols) ? x[(long)r * ldx + c] : (bf16)0.0f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < ldy) y[(long)c * ldy + r] = tile[tx][i];
  }
}

}  // namespace

extern "C" int dc_latent_scale_fwd(const void* x, int ldx, long long pixels, float scale, void* y, void* stream) {
  if (!x || !y || pixels <= 0 || !(scale > 0.0f)) return DC_ERR_ARG;
  hipLaunchKernelGGL(latent_scale_fwd_kernel, grid_for(pixels), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, ldx,
                     (long)pixels, scale, (bf16*)y);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_latent_scale_bwd(const void* dy, int lddy, long long pixels, float scale, const float* coef,
                                   const int* step, void* gx_direct, void* dv, void* stream) {
  if (!dy || !coef || !step || !gx_direct || !dv || pixels <= 0 || !(scale > 0.0f)) return DC_ERR_ARG;
  hipLaunchKernelGGL(latent_scale_bwd_kernel, grid_for(pixels), dim3(256), 0, (hipStream_t)stream, (const bf16*)dy,
                     lddy, (long)pixels, scale, coef, step, (bf16*)gx_direct, (bf16*)dv);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_softmax_rows(const void* s, int lds, long long rows, int cols, float scale, void* p, int ldp,
                               void* stream) {
  if (!s || !p || rows <= 0 || cols <= 0 || lds < cols || ldp < cols) return DC_ERR_ARG;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)rows), dim3(kSmThreads), 0, (hipStream_t)stream,
                     (const bf16*)s, lds, cols, scale, (bf16*)p, ldp);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_softmax_rows_bwd(const void* p, int ldp, const void* dp, int lddp, long long rows, int cols,
                                   float scale, void* ds, int ldds, void* stream) {
  if (!p || !dp || !ds || rows <= 0 || cols <= 0 || ldp < cols || lddp < cols || ldds < cols) return DC_ERR_ARG;
  hipLaunchKernelGGL(softmax_rows_bwd_kernel, dim3((unsigned)rows), dim3(kSmThreads), 0, (hipStream_t)stream,
                     (const bf16*)p, ldp, (const bf16*)dp, lddp, cols, scale, (bf16*)ds, ldds);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

extern "C" int dc_transpose(const void* x, int ldx, int rows, int cols, void* y, int ldy, void* stream) {
  if (!x || !y || rows <= 0 || cols <= 0 || ldx < cols || ldy < rows) return DC_ERR_ARG;
  const dim3 grid((cols + 63) / 64, (ldy + 63) / 64);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, ldx, rows, cols,
                     (bf16*)y, ldy);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// Depth-completion evaluation metrics (analyze.py:233-290, utils.py:692-740) on gfx950.
//
// One batch of dense predictions against the 8-bit sparse LiDAR maps: the valid mask is taken
// before clamping (sparse > 0), both maps are clamped to [min_depth, max_depth], and for the whole
// batch ("overall") and for every depth bin [lo, hi] (inclusive both ends, on the clamped sparse value,
// as the reference bins it) the kernel returns sum |d - s|, sum (d - s)^2 and the point count.
// MAE = sum|e| / n and RMSE = sqrt(sum e^2 / n) follow on the host.  Deterministic: per-thread fp64
// sums over a grid-stride range, a fixed-order block fold, then one block folding the block partials
// in block order.  Bins are handled 16 per pass (the per-thread accumulators stay in registers).
#include "common.h"
#include "../../include/dcamd.h"

namespace {

constexpr int kBinsPerPass = 16;
constexpr int kThreads = 256;
constexpr int kMaxBlocks = 1024;

// fixed-order block sum of a double (LDS tree over 256 threads)
__device__ double block_sum_d(double v, double* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

// part[blk][1 + kBinsPerPass][3]: slot 0 overall (pass 0 only), slots 1.. the pass's bins
__global__ __launch_bounds__(kThreads) void depth_metrics_kernel(const float* dense, const float* sparse, long total,
                                                                 float lo, float hi, const float* bins, int b0,
                                                                 int nb, double* part) {
  __shared__ double sh[kThreads];
  double acc[1 + kBinsPerPass][3];
#pragma unroll
  for (int b = 0; b <= kBinsPerPass; ++b) acc[b][0] = acc[b][1] = acc[b][2] = 0.0;
  float blo[kBinsPerPass], bhi[kBinsPerPass];
#pragma unroll
  for (int b = 0; b < kBinsPerPass; ++b) {
    blo[b] = b < nb ? bins[(b0 + b) * 2] : 1.0f;
    bhi[b] = b < nb ? bins[(b0 + b) * 2 + 1] : 0.0f;  // empty interval past the last bin
  }
  for (long i = (long)blockIdx.x * kThreads + threadIdx.x; i < total; i += (long)gridDim.x * kThreads) {
    const float s = sparse[i];
    if (!(s > 0.0f)) continue;
    const float sc = fminf(fmaxf(s, lo), hi);
    const float dc = fminf(fmaxf(dense[i], lo), hi);
    const float e = dc - sc;
    const double ae = (double)fabsf(e), se = (double)(e * e);
    acc[0][0] += ae;
    acc[0][1] += se;
    acc[0][2] += 1.0;
#pragma unroll
    for (int b = 0; b < kBinsPerPass; ++b) {
      if (sc >= blo[b] && sc <= bhi[b]) {
        acc[1 + b][0] += ae;
        acc[1 + b][1] += se;
        acc[1 + b][2] += 1.0;
      }
    }
  }
  double* out = part + (long)blockIdx.x * (1 + kBinsPerPass) * 3;
#pragma unroll
  for (int b = 0; b <= kBinsPerPass; ++b)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double t = block_sum_d(acc[b][k], sh);
      if (threadIdx.x == 0) out[b * 3 + k] = t;
    }
}

// res[(1 + nbins)][3]: overall, then bins b0 .. b0 + nb - 1 (pass 0 also writes the overall row)
__global__ void depth_metrics_fold_kernel(const double* part, int nblk, int b0, int nb, double* res) {
  const int slot = threadIdx.x / 3, k = threadIdx.x % 3;
  if (slot > kBinsPerPass || (slot == 0 && b0 != 0) || (slot > 0 && slot > nb)) return;
  double t = 0.0;
  for (int blk = 0; blk < nblk; ++blk) t += part[((long)blk * (1 + kBinsPerPass) + slot) * 3 + k];
  const int row = slot == 0 ? 0 : 1 + b0 + slot - 1;
  res[row * 3 + k] = t;
}

}  // namespace

extern "C" long long dc_depth_metrics_ws_bytes(void) {
  return (long long)kMaxBlocks * (1 + kBinsPerPass) * 3 * (long long)sizeof(double);
}

extern "C" int dc_depth_metrics(const float* dense, const float* sparse, long long total, float min_depth,
                                float max_depth, const float* bins, int nbins, double* ws, double* res,
                                void* stream) {
  if (!dense || !sparse || !ws || !res || total <= 0 || nbins < 0 || (nbins > 0 && !bins)) return DC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int nblk = (int)min((long long)kMaxBlocks, (total + kThreads - 1) / kThreads);
  for (int b0 = 0; b0 == 0 || b0 < nbins; b0 += kBinsPerPass) {
    const int nb = min(kBinsPerPass, nbins - b0);
    hipLaunchKernelGGL(depth_metrics_kernel, dim3(nblk), dim3(kThreads), 0, st, dense, sparse, (long)total, min_depth,
                       max_depth, bins, b0, nb > 0 ? nb : 0, ws);
    hipLaunchKernelGGL(depth_metrics_fold_kernel, dim3(1), dim3(3 * (1 + kBinsPerPass)), 0, st, ws, nblk, b0,
                       nb > 0 ? nb : 0, res);
  }
  DC_CHECK_LAUNCH();
  return DC_OK;
}

// Seed ensemble of the guided sampler (BASELINE.json config C5: 10 seeds per frame, mean, affine fit).
//
// The S seeds of a frame run as S frames of one batched guided call (frames never interact,
// marigold_dc.py:877), each with its own initial noise (dc_latent_init, noise_frames = nb).  This file
// folds their dense outputs: the per-pixel mean over the seeds, then compute_affine_params
// (marigold_dc.py:53-128) of the mean against the sparse guide over its valid pixels (guide > 0),
// applied to the whole mean map.  HBM-bound: the S dense maps are read once, the fitted map is written
// once and read back once for the centred sums and once for the apply.
//
// Three launches, deterministic (fixed-order folds of per-block fp64 partials, no atomics):
//   1. mean over seeds -> out, per-block partials (count, sum a, sum g) over the masked pixels
//   2. every block folds its frame's partials (means), then partials of the centred sums
//      sum (a - mean_a)^2 and sum (a - mean_a)(g - mean_g) (the reference's centring, :111-121)
//   3. every block folds those, forms scale = cov / (var + 1e-7), shift = mean_g - scale mean_a (:124-125)
//      and applies them in place.
#include "common.h"
#include "../../include/dcamd.h"

namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;                        // pixels per thread per block
constexpr long kPix = (long)kThreads * kItems;    // pixels per block

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide fp64 sum in a fixed order (lane order within a wave, then wave order); every thread gets it
__device__ __forceinline__ double block_sum_d(double v, double* scratch) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) t += scratch[i];
  return t;
}

// fold K consecutive doubles per block over nblk blocks (fixed order: strided per lane, then the block sum)
template <int K>
__device__ __forceinline__ void fold_partials(const double* part, int nblk, double* out, double* scratch) {
  double acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.0;
  for (int b = threadIdx.x; b < nblk; b += kThreads)
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] += part[(long)b * K + k];
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = block_sum_d(acc[k], scratch);
}

__global__ __launch_bounds__(kThreads) void ens_mean_kernel(const float* dense, int seeds, long hw, const float* guide,
                                                            float* out, double* part1, int nblk) {
  __shared__ double scratch[kThreads / 64];
  const int f = blockIdx.y, b = blockIdx.x;
  const float inv = 1.0f / (float)seeds;
  double n = 0.0, sa = 0.0, sg = 0.0;
  const long base = (long)b * kPix;
#pragma unroll 4
  for (int it = 0; it < kItems; ++it) {
    const long p = base + (long)it * kThreads + threadIdx.x;
    if (p >= hw) break;
    float s = 0.0f;
    for (int k = 0; k < seeds; ++k) s += dense[((long)f * seeds + k) * hw + p];   // torch.stack(...).mean(0) order
    const float a = s * inv;
    out[(long)f * hw + p] = a;
    const float g = guide[(long)f * hw + p];
    if (g > 0.0f) {
      n += 1.0;
      sa += a;
      sg += g;
    }
  }
  n = block_sum_d(n, scratch);
  sa = block_sum_d(sa, scratch);
  sg = block_sum_d(sg, scratch);
  if (threadIdx.x == 0) {
    double* q = part1 + ((long)f * nblk + b) * 3;
    q[0] = n;
    q[1] = sa;
    q[2] = sg;
  }
}

__global__ __launch_bounds__(kThreads) void ens_centred_kernel(const float* out, long hw, const float* guide,
                                                               const double* part1, double* part2, int nblk) {
  __shared__ double scratch[kThreads / 64];
  const int f = blockIdx.y, b = blockIdx.x;
  double s1[3];
  fold_partials<3>(part1 + (long)f * nblk * 3, nblk, s1, scratch);
  const double ma = s1[0] > 0.0 ? s1[1] / s1[0] : 0.0, mg = s1[0] > 0.0 ? s1[2] / s1[0] : 0.0;
  double va = 0.0, cv = 0.0;
  const long base = (long)b * kPix;
#pragma unroll 4
  for (int it = 0; it < kItems; ++it) {
    const long p = base + (long)it * kThreads + threadIdx.x;
    if (p >= hw) break;
    const float g = guide[(long)f * hw + p];
    if (g > 0.0f) {
      const double da = (double)out[(long)f * hw + p] - ma;
      va += da * da;
      cv += da * ((double)g - mg);
    }
  }
  va = block_sum_d(va, scratch);
  cv = block_sum_d(cv, scratch);
  if (threadIdx.x == 0) {
    double* q = part2 + ((long)f * nblk + b) * 2;
    q[0] = va;
    q[1] = cv;
  }
}

__global__ __launch_bounds__(kThreads) void ens_apply_kernel(float* out, long hw, const double* part1,
                                                             const double* part2, int nblk, float* affine) {
  __shared__ double scratch[kThreads / 64];
  const int f = blockIdx.y, b = blockIdx.x;
  double s1[3], s2[2];
  fold_partials<3>(part1 + (long)f * nblk * 3, nblk, s1, scratch);
  fold_partials<2>(part2 + (long)f * nblk * 2, nblk, s2, scratch);
  const double ma = s1[1] / s1[0], mg = s1[2] / s1[0];
  const double scale = s2[1] / (s2[0] + 1e-7);          // EPSILON, marigold_dc.py:20, 124
  const double shift = mg - scale * ma;
  const float sc = (float)scale, sh = (float)shift;
  if (b == 0 && threadIdx.x == 0 && affine) {
    affine[2 * f] = sc;
    affine[2 * f + 1] = sh;
  }
  const long base = (long)b * kPix;
#pragma unroll 4
  for (int it = 0; it < kItems; ++it) {
    const long p = base + (long)it * kThreads + threadIdx.x;
    if (p >= hw) break;
    out[(long)f * hw + p] = out[(long)f * hw + p] * sc + sh;
  }
}

}  // namespace

extern "C" long long dc_ensemble_ws_bytes(int frames, long long hw) {
  if (frames <= 0 || hw <= 0) return 0;
  const long nblk = (hw + kPix - 1) / kPix;
  return (long long)frames * nblk * 5 * (long long)sizeof(double);
}

extern "C" int dc_ensemble_fit(const float* dense, int frames, int seeds, long long hw, const float* guide, float* out,
                               float* affine, void* ws, long long ws_bytes, void* stream) {
  if (!dense || !guide || !out || !ws || frames <= 0 || seeds <= 0 || hw <= 0) return DC_ERR_ARG;
  if (frames > 65535 || ws_bytes < dc_ensemble_ws_bytes(frames, hw)) return DC_ERR_ARG;
  if ((uintptr_t)ws & 7) return DC_ERR_ALIGN;
  const int nblk = (int)((hw + kPix - 1) / kPix);
  double* part1 = (double*)ws;
  double* part2 = part1 + (long)frames * nblk * 3;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(nblk, frames);
  hipLaunchKernelGGL(ens_mean_kernel, grid, dim3(kThreads), 0, s, dense, seeds, (long)hw, guide, out, part1, nblk);
  DC_CHECK_LAUNCH();
  hipLaunchKernelGGL(ens_centred_kernel, grid, dim3(kThreads), 0, s, (const float*)out, (long)hw, guide,
                     (const double*)part1, part2, nblk);
  DC_CHECK_LAUNCH();
  hipLaunchKernelGGL(ens_apply_kernel, grid, dim3(kThreads), 0, s, out, (long)hw, (const double*)part1,
                     (const double*)part2, nblk, affine);
  DC_CHECK_LAUNCH();
  return DC_OK;
}

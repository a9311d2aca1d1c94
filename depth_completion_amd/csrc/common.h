// Shared device helpers for the gfx950 (CDNA4) kernels of the Marigold-DC guided sampler.
// Storage type is bf16 (``__bf16``) with fp32 accumulation everywhere; layouts are NHWC
// ("pixel rows" of C contiguous channels), token rows [T][C] for the transformer path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DC_LDS __attribute__((address_space(3)))

// Status codes returned by every C-ABI entry point (mapped to ValueError / RuntimeError in Python).
enum {
  DC_OK = 0,
  DC_ERR_ARG = 1,      // invalid shape / argument
  DC_ERR_LAUNCH = 2,   // hipGetLastError after launch
  DC_ERR_ALIGN = 3,    // pointer / leading-dimension alignment violated
};

#define DC_CHECK_LAUNCH()                                  \
  do {                                                     \
    if (hipGetLastError() != hipSuccess) return DC_ERR_LAUNCH; \
  } while (0)

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

__device__ __forceinline__ float silu_f(float y) { return y / (1.0f + __expf(-y)); }
// d/dy silu(y) = s * (1 + y * (1 - s)), s = sigmoid(y)
__device__ __forceinline__ float silu_grad(float y) {
  float s = 1.0f / (1.0f + __expf(-y));
  return s * (1.0f + y * (1.0f - s));
}

// exact GELU (F.gelu, approximate="none") and its derivative, fp32
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block reduction over up to 1024 threads, result broadcast to all threads.
// `scratch` must hold >= 16 floats and is reused, callers separate calls with the returned value.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float t = (l < nw) ? scratch[l] : 0.0f;
  t = wave_sum(t);
  return t;
}

__device__ __forceinline__ void load8(const bf16* p, float* f) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
__device__ __forceinline__ void store8(bf16* p, const float* f) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)f[i];
  *reinterpret_cast<bf16x8*>(p) = v;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

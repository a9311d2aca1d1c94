// Order-independent GroupNorm statistics accumulators (include/dcamd.h dc_gn_fuse), shared by the conv epilogues
// that add to them (conv_gemm.hip) and the one-pass GroupNorm kernels that read them (norms.hip).
//
// A quantity is kGnWords int64 words: 8 limbs of a fixed-point integer whose LSB is 2^-120 (limb j holds bits
// [32 j, 32 j + 32) of every contribution, with 32 bits of headroom for carries) and a count of non-finite
// contributions.  A finite fp32 x = m 2^(e - 150) (m the 24-bit significand, e the biased exponent) with e >= 30
// adds m << (e - 30) to at most two adjacent limbs; |x| < 2^-97 is dropped.  Integer addition commutes, so the
// accumulated value is the exact sum of the contributions whatever order the tiles arrive in: the statistics are
// bitwise reproducible without a fixed-order fold.  The contributions themselves are not the elements: each block
// first folds its tile's per-lane / per-channel sums in fp32 (a fixed order, so deterministic, but rounded), and
// only those block partials are summed exactly -- accurate to the fp32 partials, not exact over the elements.
#pragma once
#include "common.h"

constexpr int kGnWords = 9;              // per quantity
constexpr int kGnPair = 2 * kGnWords;    // per (frame, group): the two quantities
// The accumulators exist in kGnReplicas copies ([replica][frame][group][2][kGnWords]); a producing block adds to
// copy (block id mod kGnReplicas) and readers sum the copies (integers: still exact).  The atomics of every tile
// of a launch otherwise land on the same few words per group, which serialises them at the memory-side atomic
// units.
constexpr int kGnReplicas = 4;

// add x to the quantity at q (vector atomics on global memory)
__device__ __forceinline__ void gn_acc_add(unsigned long long* q, float x) {
  const unsigned b = __float_as_uint(x);
  const int e = (int)((b >> 23) & 0xffu);
  if (e == 0xff) {
    atomicAdd(q + 8, 1ull);
    return;
  }
  if (e < 30) return;
  const int p = e - 30;   // 0 .. 224: limb p / 32, shift p % 32 (p = 224 has shift 0, so limb 8 is never reached)
  const unsigned long long m = (unsigned long long)((b & 0x7fffffu) | 0x800000u) << (p & 31);
  unsigned long long lo = m & 0xffffffffull, hi = m >> 32;
  if (b >> 31) {
    lo = 0ull - lo;
    hi = 0ull - hi;
  }
  unsigned long long* w = q + (p >> 5);
  if (lo) atomicAdd(w, lo);
  if (hi) atomicAdd(w + 1, hi);
}

// the value of a quantity summed over its replicas (rstride: words per replica; NaN if a non-finite value was added)
__device__ __forceinline__ double gn_acc_read(const unsigned long long* q0, long rstride) {
  unsigned long long q[kGnWords];
#pragma unroll
  for (int j = 0; j < kGnWords; ++j) q[j] = 0;
#pragma unroll
  for (int r = 0; r < kGnReplicas; ++r)
#pragma unroll
    for (int j = 0; j < kGnWords; ++j) q[j] += q0[r * rstride + j];   // integer sums: exact, order-free
  if (q[8]) return __builtin_nan("");
  unsigned d[8];
  long long carry = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long long v = (long long)q[j] + carry;   // |q[j]| < 2^63: < 2^31 contributions of < 2^32 each
    d[j] = (unsigned)v;
    carry = v >> 32;                                // arithmetic: floor division
  }
  // value = (carry 2^256 + sum_j d_j 2^(32 j)) 2^-120 with carry in {0, -1} (|sum| < 2^136)
  const bool neg = carry < 0;
  if (neg) {   // two's complement negation of the 256-bit digit string
    unsigned long long c = 1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned long long t = (unsigned long long)(~d[j]) + c;
      d[j] = (unsigned)t;
      c = t >> 32;
    }
  }
  double r = 0.0;
#pragma unroll
  for (int j = 7; j >= 0; --j) r += ldexp((double)d[j], 32 * j - 120);
  return neg ? -r : r;
}

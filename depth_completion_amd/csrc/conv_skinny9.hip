// The weight-streaming skinny conv / linear kernels with 9 taps (conv_skinny.h); their own translation unit
// so that the variants compile in parallel with the rest of dc_conv_gemm.
#include "conv_gemm_impl.h"

namespace {
#include "conv_skinny.h"
}  // namespace

int conv_launch_skinny9(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  return launch_skinny_idx<9>(i, p, splits, s);
}

int conv_launch_resident(int i, ConvGemmParams& p, int bpc, hipStream_t s) { return launch_resident_idx(i, p, bpc, s); }

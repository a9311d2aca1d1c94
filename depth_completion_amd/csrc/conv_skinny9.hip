// The weight-streaming skinny conv / linear kernels with 9 taps (conv_skinny.h); their own translation unit
// so that the variants compile in parallel with the rest of dc_conv_gemm.
#include "conv_gemm_impl.h"

namespace {
#include "conv_skinny.h"
}  // namespace

int conv_launch_skinny9_gn(int i, ConvGemmParams& p, int splits, hipStream_t s);    // conv_skinny9_gn.hip
int conv_launch_skinny9_gnb(int i, ConvGemmParams& p, int splits, hipStream_t s);   // conv_skinny9_gnb.hip

int conv_launch_skinny9(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  if (p.gn.mode == 1) return conv_launch_skinny9_gn(i, p, splits, s);
  if (p.gn.mode == 2) return conv_launch_skinny9_gnb(i, p, splits, s);
  return launch_skinny_idx<9, 0>(i, p, splits, s);
}

int conv_launch_resident(int i, ConvGemmParams& p, int bpc, hipStream_t s) { return launch_resident_idx(i, p, bpc, s); }

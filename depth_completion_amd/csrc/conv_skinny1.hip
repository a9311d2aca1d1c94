// The weight-streaming skinny conv / linear kernels with 1 tap (conv_skinny.h); their own translation unit
// so that the variants compile in parallel with the rest of dc_conv_gemm.
#include "conv_gemm_impl.h"

namespace {
#include "conv_skinny.h"
}  // namespace

int conv_launch_skinny1_gn(int i, ConvGemmParams& p, int splits, hipStream_t s);    // conv_skinny1_gn.hip
int conv_launch_skinny1_gnb(int i, ConvGemmParams& p, int splits, hipStream_t s);   // conv_skinny1_gnb.hip

int conv_launch_skinny1(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  if (p.gn.mode == 1) return conv_launch_skinny1_gn(i, p, splits, s);
  if (p.gn.mode == 2) return conv_launch_skinny1_gnb(i, p, splits, s);
  return launch_skinny_idx<1, 0>(i, p, splits, s);
}

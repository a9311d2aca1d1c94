// The skinny kernels with 9 taps (conv_skinny.h) with fused GroupNorm statistics in their epilogues (include/dcamd.h
// dc_gn_fuse mode 2, backward sums): a translation unit of its own, compiled in parallel with the plain forms.
#include "conv_gemm_impl.h"

namespace {
#include "conv_skinny.h"
}  // namespace

int conv_launch_skinny9_gnb(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  return launch_skinny_idx<9, 2>(i, p, splits, s);
}

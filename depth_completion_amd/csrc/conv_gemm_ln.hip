// The LayerNorm-folded instantiations of the im2col conv / linear kernel (include/dcamd.h dc_ln_fuse: the rows'
// (mean, rstd) applied in the epilogue with the folded weight's column constants): a translation unit of its own,
// compiled in parallel with conv_gemm.hip.
#include "conv_gemm_impl.h"

int conv_launch_algo_ln(int algo, ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t s) {
  return launch_algo_idx<3>(algo, p, M, splits, smallc, s);
}

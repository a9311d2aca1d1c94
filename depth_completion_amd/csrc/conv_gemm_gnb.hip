// The fused GroupNorm-statistics instantiations of the conv kernels (include/dcamd.h dc_gn_fuse), mode 2 (backward: dy' and its sums):
// a translation unit of its own, compiled in parallel with conv_gemm.hip.
#include "conv_gemm_impl.h"

int conv_launch_halo_gnb(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  return launch_halo_idx<2>(i, p, splits, s);
}
int conv_launch_algo_gnb(int algo, ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t s) {
  return launch_algo_idx<2>(algo, p, M, splits, smallc, s);
}

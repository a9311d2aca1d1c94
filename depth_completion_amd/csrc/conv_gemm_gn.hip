// The fused GroupNorm-statistics instantiations of the conv kernels (include/dcamd.h dc_gn_fuse), mode 1 (forward statistics):
// a translation unit of its own, compiled in parallel with conv_gemm.hip.
#include "conv_gemm_impl.h"

int conv_launch_halo_gn(int i, ConvGemmParams& p, int splits, hipStream_t s) {
  return launch_halo_idx<1>(i, p, splits, s);
}
int conv_launch_algo_gn(int algo, ConvGemmParams& p, long M, int splits, bool smallc, hipStream_t s) {
  return launch_algo_idx<1>(algo, p, M, splits, smallc, s);
}

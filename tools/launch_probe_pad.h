// code-size padding: many large kernels in this code object
#include <hip/hip_runtime.h>
#include <utility>
template <int I>
__global__ __launch_bounds__(256) void pad_kernel(float* out, int flag) {
  if (flag != 12345) return;
  float a = out[threadIdx.x];
#pragma unroll
  for (int i = 0; i < 1500; ++i) a = a * (1.0001f + I * 1e-7f) + (float)(i ^ I);
  out[threadIdx.x] = a;
}
template <int I>
void launch_one() {
  hipLaunchKernelGGL(pad_kernel<I>, dim3(1), dim3(1), 0, 0, nullptr, 0);
}
template <int... I>
void reg(std::integer_sequence<int, I...>) {
  (launch_one<I>(), ...);
}
void pad_all() { reg(std::make_integer_sequence<int, 600>{}); }

// Host cost of kernel launches on this ROCm stack: eager hipLaunchKernelGGL vs hipGraphLaunch of a
// captured chain of N nodes, and the GPU time of the same chain.
// Build: hipcc -O2 --offload-arch=gfx950 tools/launch_bench.hip -o /tmp/launch_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void tiny(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.0f;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 844;
  float* buf;
  hipMalloc(&buf, 1 << 20);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, buf, 65536);
  hipStreamSynchronize(s);

  double t0 = now_ms();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, buf, 65536);
  double t1 = now_ms();
  hipStreamSynchronize(s);
  double t2 = now_ms();
  printf("eager: %d launches host %.3f ms (%.2f us/launch), to completion %.3f ms (%.2f us/kernel)\n", N, t1 - t0,
         (t1 - t0) * 1e3 / N, t2 - t0, (t2 - t0) * 1e3 / N);

  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, s, buf, 65536);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  for (int rep = 0; rep < 3; ++rep) {
    t0 = now_ms();
    hipGraphLaunch(ge, s);
    t1 = now_ms();
    hipStreamSynchronize(s);
    t2 = now_ms();
    printf("graph: %d nodes host %.3f ms (%.2f us/node), to completion %.3f ms (%.2f us/node)\n", N, t1 - t0,
           (t1 - t0) * 1e3 / N, t2 - t0, (t2 - t0) * 1e3 / N);
  }
  t0 = now_ms();
  for (int rep = 0; rep < 10; ++rep) hipGraphLaunch(ge, s);
  t1 = now_ms();
  hipStreamSynchronize(s);
  t2 = now_ms();
  printf("graph x10 back-to-back: host %.3f ms, to completion %.3f ms (%.2f us/node)\n", t1 - t0, t2 - t0,
         (t2 - t0) * 1e3 / (10.0 * N));
  return 0;
}

// Per-launch floor of libdcamd's dc_conv_gemm captured in a hipGraph from C++ (no Python / torch), next to dc_silu:
// 40 back-to-back launches, device time per launch.  DC_HALO_DIAG=128 makes the conv kernel return at entry.
// Build: hipcc -O2 --offload-arch=gfx950 tools/launch_probe_lib.cpp -Ldepth_completion_amd -ldcamd
//        -Wl,-rpath,'$ORIGIN/../depth_completion_amd' -o tools/launch_probe_lib.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>

#include "../include/dcamd.h"

static float timed(const char* name, hipStream_t s, const std::function<void()>& launch) {
  const int N = 40;
  launch();
  hipStreamSynchronize(s);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < N; ++i) launch();
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0, s);
    hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  printf("%-52s %7.2f us per launch\n", name, best * 1000.0f / N);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return best;
}

int main() {
  const int M = 6912, N = 320, K = 64;
  void *x, *w, *y, *ws;
  hipMalloc(&x, (size_t)M * K * 2);
  hipMalloc(&w, (size_t)N * K * 2);
  hipMalloc(&y, (size_t)M * N * 2);
  const long long wsb = 96ll << 20;
  hipMalloc(&ws, wsb);
  hipMemset(x, 0, (size_t)M * K * 2);
  hipMemset(w, 0, (size_t)N * K * 2);
  hipMemset(ws, 0, wsb);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  timed("dc_silu 4096", s, [&] { dc_silu(y, 4096, y, s); });
  dc_conv_desc d;
  memset(&d, 0, sizeof d);
  d.x = x;
  d.ldx = K;
  d.nb = 1;
  d.hin = 1;
  d.win = M;
  d.cin = K;
  d.hout = 1;
  d.wout = M;
  d.kh = d.kw = 1;
  d.stride = 1;
  d.pad = 0;
  d.w = w;
  d.ktot = K;
  d.cout = N;
  d.y = y;
  d.ldy = N;
  d.ws = (float*)ws;
  d.ws_bytes = wsb;
  d.splitk = 1;
  for (int algo : {13, 12}) {
    d.algo = algo;
    for (const char* diag : {"128", "0"}) {
      setenv("DC_HALO_DIAG", diag, 1);
      char n[96];
      snprintf(n, sizeof n, "dc_conv_gemm K=64 algo %d diag %s", algo, diag);
      timed(n, s, [&] {
        if (dc_conv_gemm(&d, s)) printf("error\n");
      });
    }
  }
  return 0;
}

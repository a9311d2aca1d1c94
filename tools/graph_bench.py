"""Host cost of torch.cuda.CUDAGraph.replay() for graphs of libdcamd launches (GPU).

Compares a graph of N tiny dc_silu kernels with and without hipMemsetAsync nodes, to find what
makes the captured guided step slow to enqueue.
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402


def bench(fn, label):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{label}: host {1e3 * (t1 - t0) / 10:.3f} ms/replay, total {1e3 * (t2 - t0) / 10:.3f} ms/replay",
          flush=True)


def main():
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    x = torch.randn(65536, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    z = torch.zeros(4096, device=dev)
    N = 844
    bench(lambda: [ops.silu(ctx, x, y) for _ in range(N)], f"{N} kernels")
    bench(lambda: [ops.silu(ctx, x, y) if i % 50 else ops.memset(ctx, z) for i in range(N)],
          f"{N} kernels incl. {N // 50 + 1} memsets")
    bench(lambda: [ops.silu(ctx, x, y) if i % 50 else z.zero_() for i in range(N)],
          f"{N} kernels incl. {N // 50 + 1} torch fills")


if __name__ == "__main__":
    main()

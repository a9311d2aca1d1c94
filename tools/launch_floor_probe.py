"""Per-launch floor of a hipGraph-replayed chain of dependent tiny kernels (GPU).

Prints the replay time per node for a 512-node chain of one-element in-place adds: the fixed cost every kernel
node of the guided step pays (dispatch, wave launch, end-of-kernel release) whatever its work.  Used to A/B HIP
runtime environment settings (tools/ab/r06o.sh).
"""
import json
import os

import torch

dev = torch.device("cuda:0")
x = torch.zeros(1, device=dev)
n = 512
x.add_(1.0)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(n):
        x.add_(1.0)
g.replay()
torch.cuda.synchronize()
best = float("inf")
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) * 1e3 / n)
env = {k: os.environ[k] for k in ("HIP_FORCE_DEV_KERNARG", "DEBUG_CLR_GRAPH_PACKET_CAPTURE") if k in os.environ}
print(json.dumps({"us_per_node": round(best, 3), "nodes": n, "env": env}))

"""Probe (GPU, timing only): LayerNorm fwd / bwd and the one-pass GroupNorm apply (fused-statistics form) at the
UNet's shapes under the launch-shape knobs DC_LN_WPB (waves per LayerNorm block), DC_GN_T (threads per GroupNorm
apply block, rounded to whole 8-channel rows) and DC_GN_BPF (GroupNorm apply blocks per frame); each call timed
inside a 20-call graph captured under the setting.  The knobs existed in norms.hip only for this probe (round 5,
profiles/r05ac/: the committed shapes won); without them every setting times the committed shape.  Args: none."""
import os
import sys

import torch

sys.path.insert(0, ".")
from depth_completion_amd import ops  # noqa: E402
from depth_completion_amd.ops import Ctx  # noqa: E402

dev = torch.device("cuda:0")
ctx = Ctx(dev)


def graph_time(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def r(*s):
    return torch.randn(*s, device=dev).to(torch.bfloat16)


for rows, c in [(6912, 320), (1728, 640), (432, 1280), (108, 1280)]:
    x, dy, add = r(rows, c), r(rows, c), r(rows, c)
    y, dx = torch.empty_like(x), torch.empty_like(x)
    g, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    st = torch.empty(rows, 2, device=dev)
    ops.layernorm(ctx, x, rows, c, g, b, 1e-5, y, st)
    out = []
    for wpb in ("1", "2", "4", "8", "16"):
        os.environ["DC_LN_WPB"] = wpb
        tf = graph_time(lambda: ops.layernorm(ctx, x, rows, c, g, b, 1e-5, y, st))
        tb = graph_time(lambda: ops.call("dc_layernorm_bwd", ops.P(x), ops.LD(x), rows, c, g.data_ptr(), st.data_ptr(),
                                         ops.P(dy), ops.LD(dy), ops.P(dx), ops.LD(dx), ops.P(add), ops.LD(add),
                                         ctx.stream))
        out.append(f"wpb {wpb}: {tf:.1f}/{tb:.1f}")
    os.environ.pop("DC_LN_WPB")
    print(f"LN rows={rows} C={c} (fwd/bwd us): " + "  ".join(out), flush=True)

for nb, hw, c in [(1, 6912, 320), (1, 6912, 640), (1, 1728, 640), (1, 1728, 1280)]:
    x = r(nb * hw, c)
    g, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    y, dyp, dx, add = torch.empty_like(x), r(nb * hw, c), torch.empty_like(x), r(nb * hw, c)
    st = torch.zeros(nb, 32, 2, device=dev)
    st[..., 1] = 1.0
    acc = torch.zeros(ops.gn_acc_words(nb), dtype=torch.int64, device=dev)
    out = []
    for t, bpf in (("256", "1024"), ("512", "1024"), ("1024", "1024"), ("256", "512"), ("256", "2048"),
                   ("512", "512")):
        os.environ["DC_GN_T"], os.environ["DC_GN_BPF"] = t, bpf
        tf = graph_time(lambda: ops.groupnorm_acc(ctx, x, nb, hw, c, g, b, 1e-5, True, acc, y, st))
        tb = graph_time(lambda: ops.groupnorm_bwd_acc(ctx, x, nb, hw, c, g, st, acc, dyp, dx, add1=add))
        out.append(f"T{t}/B{bpf}: {tf:.1f}/{tb:.1f}")
    os.environ.pop("DC_GN_T")
    os.environ.pop("DC_GN_BPF")
    print(f"GN apply hw={hw} C={c} (fwd/bwd us): " + "  ".join(out), flush=True)

"""Self-attention outputs on seeded inputs, saved for a bitwise comparison of two library builds (GPU).

    DC_LIB=ab/lib_a.so python tools/attn_bits.py out_a.pt ; python tools/attn_bits.py out_b.pt
    python tools/attn_bits.py --compare out_a.pt out_b.pt
Shapes: the UNet levels' (frames, tokens, heads) at batch 1 (level 0 takes the stream-K backward), a batch-2 level 1,
and ragged token counts; forward (O, lse) and backward (dQKV).
"""
import sys

import torch

sys.path.insert(0, ".")

CASES = [(1, 6912, 5), (1, 1728, 10), (1, 432, 20), (1, 108, 20), (2, 1728, 10), (1, 1000, 5), (1, 77, 20)]


def run(path):
    from depth_completion_amd import ops
    from depth_completion_amd.ops import Ctx
    dev = torch.device("cuda:0")
    ctx = Ctx(dev)
    out = {}
    for nb, t, heads in CASES:
        g = torch.Generator(device="cpu").manual_seed(nb * 1000 + t)
        c = 64 * heads
        qkv = torch.randn(nb * t, 3 * c, generator=g).to(dev).to(torch.bfloat16)
        o = torch.empty(nb * t, c, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(nb, heads, t, device=dev)
        ops.attn_fwd(ctx, qkv, nb, t, heads, o, lse)
        dout = torch.randn(nb * t, c, generator=g).to(dev).to(torch.bfloat16)
        delta = torch.empty(2, nb, heads, t, device=dev)
        dqkv = torch.empty_like(qkv)
        ops.attn_bwd(ctx, qkv, o, dout, lse, nb, t, heads, delta, dqkv)
        torch.cuda.synchronize()
        for k, v in dict(o=o, lse=lse, dqkv=dqkv).items():
            out[f"{nb}_{t}_{k}"] = v.cpu()
    torch.save(out, path)
    print(f"saved {len(out)} tensors to {path}")


def compare(a, b):
    ta, tb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    key = lambda v: v.view(torch.int16) if v.dtype == torch.bfloat16 else v  # noqa: E731
    bad = [k for k in ta if not torch.equal(key(ta[k]), key(tb[k]))]
    print(f"{len(ta)} tensors, {len(bad)} differ: {bad}")
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])

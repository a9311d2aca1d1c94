"""Diagnose batch-vs-single differences of the HIP pipeline (full UNet, C2 shape).

Runs frame 0 alone, inside batches of 2 and 8, eager and graph-replayed, with and without the sparse-aware
decode, and prints the latent / dense relative differences to the first single run.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from test_gpu_pipeline import synth_inputs  # noqa: E402

from depth_completion_amd.config import MARIGOLD_V1  # noqa: E402
from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline  # noqa: E402
from depth_completion_amd import synthetic  # noqa: E402

dev = torch.device("cuda:0")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


usd, vsd, emb = synthetic.unet_state_dict(MARIGOLD_V1), synthetic.taesd_state_dict(), synthetic.text_embedding()
imgs, sparses = synth_inputs(8, 576, 768, 500, seed=41)
noise = torch.randn((1, 4, 72, 96), generator=torch.Generator().manual_seed(2024), dtype=torch.bfloat16)
kw = dict(norm="const", steps=steps, resolution=768, init_noise=noise)


def run(pipe, n):
    d, l = pipe(imgs[:n].to(dev), sparses[:n].to(dev), 120.0, **kw)
    torch.cuda.synchronize()
    return d[:1].cpu(), l[:1].cpu()




def diag_replay():
    """graph replay after other calls on the same pipeline (frame B, then a batch of 8) vs fresh pipelines"""
    os.environ["DC_SPARSE_DECODE"] = "0"
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)

    def one(p, i):
        d, l = p(imgs[i:i + 1].to(dev), sparses[i:i + 1].to(dev), 120.0, **kw)
        torch.cuda.synchronize()
        return d.cpu(), l.cpu()

    a = one(pipe, 0)
    b = one(pipe, 1)
    fresh = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    bf = one(fresh, 1)
    del fresh
    print(f"replay frame1 vs fresh: lat {rel(b[1], bf[1]):.3e}", flush=True)
    a2 = one(pipe, 0)
    print(f"replay frame0 again vs first: lat {rel(a2[1], a[1]):.3e}", flush=True)
    run(pipe, 2)
    c = one(pipe, 0)
    print(f"after batch-2 call, frame0 vs first: lat {rel(c[1], a[1]):.3e}", flush=True)
    pipe.ctx.ws.zero_()
    d = one(pipe, 0)
    print(f"after zeroing ws, frame0 vs first: lat {rel(d[1], a[1]):.3e}", flush=True)
    for r in pipe.unet.resnets():
        print("temb tables", {k: v.data_ptr() for k, v in r.temb_tables.items()}, r.temb_table.data_ptr())
        break


def diag_batch_steps():
    """frames must not interact: batch [f0, f0] and [f0, f1] vs single f0, eager, growing step counts"""
    os.environ["DC_SPARSE_DECODE"] = "0"
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev, use_graph=False)
    for st in (1, 2, 5):
        k = dict(kw, steps=st)
        d1, l1 = pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **k)
        i2 = torch.cat([imgs[:1], imgs[:1]]).to(dev)
        s2 = torch.cat([sparses[:1], sparses[:1]]).to(dev)
        d2, l2 = pipe(i2, s2, 120.0, **k)
        d3, l3 = pipe(imgs[:2].to(dev), sparses[:2].to(dev), 120.0, **k)
        torch.cuda.synchronize()
        print(f"steps {st}: [f0,f0] f0 vs f1 lat {rel(l2[1:], l2[:1]):.3e} | [f0,f0][0] vs single {rel(l2[:1], l1):.3e} "
              f"| [f0,f1][0] vs single {rel(l3[:1], l1):.3e} | dense [f0,f1][0] vs single {rel(d3[:1], d1):.3e}",
              flush=True)


if os.environ.get("DIAG") == "batch":
    diag_batch_steps()
    sys.exit(0)


def diag_replay2():
    """replay determinism and recapture"""
    os.environ["DC_SPARSE_DECODE"] = "0"
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    eager = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev, use_graph=False)

    def one(p, i):
        d, l = p(imgs[i:i + 1].to(dev), sparses[i:i + 1].to(dev), 120.0, **kw)
        torch.cuda.synchronize()
        return d.cpu(), l.cpu()

    e0, e1 = one(eager, 0), one(eager, 1)
    a = one(pipe, 0)
    print(f"capture call f0 vs eager f0: {rel(a[1], e0[1]):.3e}", flush=True)
    a2 = one(pipe, 0)
    a3 = one(pipe, 0)
    print(f"replay f0 vs eager f0: {rel(a2[1], e0[1]):.3e}; replay f0 twice: {rel(a3[1], a2[1]):.3e}", flush=True)
    b = one(pipe, 1)
    print(f"replay f1 vs eager f1: {rel(b[1], e1[1]):.3e}", flush=True)
    st = pipe._plans[(1, 72, 96)]
    st["graph"] = None
    b2 = one(pipe, 1)
    print(f"recaptured f1 vs eager f1: {rel(b2[1], e1[1]):.3e}", flush=True)
    # replay after the recapture, frame 0 again
    a4 = one(pipe, 0)
    print(f"replay f0 (graph captured on f1) vs eager f0: {rel(a4[1], e0[1]):.3e}", flush=True)


if os.environ.get("DIAG") == "replay2":
    diag_replay2()
    sys.exit(0)


def diag_state():
    """checksums of every plan buffer at the first replay of the capture call vs of a later replay call"""
    os.environ["DC_SPARSE_DECODE"] = "0"
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    snaps = []
    after = []
    orig = torch.cuda.CUDAGraph.replay
    state = {"armed": False}

    def bufs():
        st = pipe._plans[(1, 72, 96)]
        out = {}
        for i, t in enumerate(st["unet"].saved):
            out[f"unet{i}"] = t
        for i, t in enumerate(st["dec"].saved):
            out[f"dec{i}"] = t
        for k, v in st.items():
            if isinstance(v, torch.Tensor):
                out["st." + k] = v
        for i, t in enumerate(st.get("graph_tables") or ()):
            out[f"tab{i}"] = t
        out["step"] = pipe.ctx.step
        for j, r in enumerate(pipe.unet.resnets()):
            out[f"temb{j}"] = r.temb_table
        return out

    def snap():
        torch.cuda.synchronize()
        return {k: (float(t.double().sum()), float(t.double().abs().sum())) for k, t in bufs().items()}

    def replay(self):
        if state["armed"]:
            state["armed"] = False
            snaps.append(snap())
            r = orig(self)
            after.append(snap())
            return r
        return orig(self)

    torch.cuda.CUDAGraph.replay = replay
    for _ in range(2):
        state["armed"] = True
        pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
        torch.cuda.synchronize()
    a, b = snaps
    names = sorted(set(a) | set(b))
    ndiff = 0
    for k in names:
        if a.get(k) != b.get(k) and not k.startswith(("dec", "unet")):
            ndiff += 1
            print(f"differs at replay start: {k}: {a.get(k)} vs {b.get(k)}", flush=True)
    print(f"{ndiff} of {len(names)} buffers differ", flush=True)
    a, b = after
    order = list(bufs().keys())
    ndiff = 0
    for k in order:
        if a.get(k) != b.get(k):
            ndiff += 1
            if not k.startswith("unet") or k in ("unet0", "unet1", "unet2", "unet3"):
                print(f"differs after first replay: {k}: {a.get(k)} vs {b.get(k)}", flush=True)
    print(f"after first replay {ndiff} of {len(order)} buffers differ", flush=True)


if os.environ.get("DIAG") == "state":
    diag_state()
    sys.exit(0)


def diag_fix():
    """check the replayed tables' contents, and the sparse loss inputs, on a replay call"""
    os.environ["DC_SPARSE_DECODE"] = "0"
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    eager = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev, use_graph=False)
    e0 = eager(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
    a = pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
    st = pipe._plans[(1, 72, 96)]
    cs0 = dict(pipe._call_state)
    gt0 = [t.clone() for t in st["graph_tables"]]
    orig = torch.cuda.CUDAGraph.replay
    seen = {"n": 0}

    def replay(self):
        if seen["n"] == 0:
            torch.cuda.synchronize()
            cs = pipe._call_state
            gt = st["graph_tables"]
            c = int(cs["cnt"][0])
            for name, i in (("coef", 0), ("adam", 1), ("cnt", 4), ("params", 5)):
                print(f"{name}: table==call {torch.equal(gt[i].cpu(), cs[name].cpu())} table==first {torch.equal(gt[i].cpu(), gt0[i].cpu())}")
            for name, i in (("idx", 2), ("gval", 3)):
                print(f"{name}[:cnt]: table==call {torch.equal(gt[i][0, :c].cpu(), cs[name][0, :c].cpu())} "
                      f"table==first {torch.equal(gt[i][0, :c].cpu(), gt0[i][0, :c].cpu())}")
            print("cnt", c, "graph table ptrs", [t.data_ptr() for t in gt], flush=True)
        seen["n"] += 1
        return orig(self)

    torch.cuda.CUDAGraph.replay = replay
    b = pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
    torch.cuda.CUDAGraph.replay = orig
    torch.cuda.synchronize()
    print(f"capture vs eager {rel(a[1], e0[1]):.3e}; replay vs eager {rel(b[1], e0[1]):.3e}", flush=True)


if os.environ.get("DIAG") == "fix":
    diag_fix()
    sys.exit(0)


def diag_sync():
    """replay calls with a device synchronize before the first replay"""
    os.environ["DC_SPARSE_DECODE"] = "0"
    pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev)
    eager = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev, use_graph=False)
    e0 = eager(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
    a = pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
    orig = torch.cuda.CUDAGraph.replay
    seen = {"n": 0}

    def replay(self):
        if seen["n"] == 0:
            torch.cuda.synchronize()
            tail = pipe.ctx.ws[-(64 * 1024 // 4):].view(torch.int32)
            nz = int((tail != 0).sum())
            print(f"nonzero counters before first replay: {nz} {tail.nonzero().flatten()[:10].tolist()} "
                  f"{tail[tail != 0][:10].tolist()}", flush=True)
            if os.environ.get("ZERO_WS") == "1":
                pipe.ctx.ws.zero_()
        seen["n"] += 1
        return orig(self)

    for trial in range(3):
        torch.cuda.CUDAGraph.replay = replay
        seen["n"] = 0
        b = pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
        torch.cuda.CUDAGraph.replay = orig
        c = pipe(imgs[:1].to(dev), sparses[:1].to(dev), 120.0, **kw)
        torch.cuda.synchronize()
        print(f"trial {trial}: synced replay vs eager {rel(b[1], e0[1]):.3e}; plain replay vs eager {rel(c[1], e0[1]):.3e}",
              flush=True)


if os.environ.get("DIAG") == "sync":
    diag_sync()
    sys.exit(0)


if os.environ.get("DIAG") == "replay":
    diag_replay()
    sys.exit(0)


for graph in (True, False):
    for sd in ("1", "0"):
        os.environ["DC_SPARSE_DECODE"] = sd
        pipe = MarigoldDepthCompletionPipeline(usd, vsd, emb, unet_config=MARIGOLD_V1, device=dev, use_graph=graph)
        a = run(pipe, 1)
        b8 = run(pipe, 8)
        c = run(pipe, 1)
        b2 = run(pipe, 2)
        print(f"graph={graph} sparse_decode={sd}: single-again lat {rel(c[1], a[1]):.3e} dense {rel(c[0], a[0]):.3e} | "
              f"batch8[0] lat {rel(b8[1], a[1]):.3e} dense {rel(b8[0], a[0]):.3e} | "
              f"batch2[0] lat {rel(b2[1], a[1]):.3e} dense {rel(b2[0], a[0]):.3e}", flush=True)
        del pipe
        torch.cuda.empty_cache()

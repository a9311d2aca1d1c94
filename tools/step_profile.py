"""Per-shape conv time inside the real graph-replayed guided step (GPU, run under rocprofv3 --kernel-trace).

Run:   rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python3 tools/step_profile.py --out <descs.json>
       python tools/step_profile.py --trace <dir>/run_kernel_trace.csv --descs <descs.json>
The first form runs a C2 call (graph-replayed guided steps) and writes the conv launches of one step, in launch
order, with their shapes and chosen variants.  The second (CPU) takes the last complete step of the trace, matches
its conv dispatches (conv_gemm / conv_halo / conv_skinny (+ skinny_reduce) / conv_resident kernels) to those launches by order, and prints the time per shape
group -- the step's own cache state and launch order, unlike tools/conv_breakdown.py's warm replays.
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def record(out, batch, frame=(576, 768, 500, "uniform")):
    import threading
    import time
    import torch
    # heartbeat: under rocprofv3 --pmc every dispatch is serialised and a pass runs minutes without other output
    t_start = time.perf_counter()

    def beat():
        while True:
            time.sleep(30.0)
            print(f"step_profile: running ({time.perf_counter() - t_start:.0f} s)", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    from bench import conv_flops, synth_frame
    from depth_completion_amd import ops, synthetic
    from depth_completion_amd._lib import ConvDesc
    from depth_completion_amd.config import MARIGOLD_V1
    from depth_completion_amd.pipeline import MarigoldDepthCompletionPipeline
    dev = torch.device("cuda:0")
    pipe = MarigoldDepthCompletionPipeline(synthetic.unet_state_dict(MARIGOLD_V1, 11), synthetic.taesd_state_dict(12),
                                           synthetic.text_embedding(13, 1024), device=dev)
    h, w, npts, pattern = frame
    # C5 is a batch-10 call of one frame (the seed ensemble's shapes); other batches take distinct frames
    fr = [synth_frame(h, w, npts, 0 if batch == 10 else i, pattern) for i in range(batch)]
    imgs = torch.stack([f[0] for f in fr]).to(dev)
    sps = torch.stack([f[1] for f in fr]).to(dev)
    for _ in range(2):
        pipe(imgs, sps, 120.0, norm="const", steps=8, resolution=768)
    torch.cuda.synchronize()
    st = next(v for k, v in pipe._plans.items() if k[0] == batch)
    descs = []
    orig = ops.call

    def rec(name, *a):
        if name == "dc_conv_gemm":
            d = ConvDesc.from_buffer_copy(a[0]._obj)
            descs.append(dict(M=d.nb * d.hout * d.wout, rows=int(d.nrows) if d.rows else 0, N=d.cout,
                              K=d.kh * d.kw * d.cin, cin=d.cin, mode=d.mode, k=d.kh, stride=d.stride,
                              hw=[d.hout, d.wout], algo=int(d.algo), split=int(d.splitk), flops=conv_flops(d),
                              key=[int(v) for v in ops.conv_key(d)]))
        return orig(name, *a)

    # the captured step's launch sequence: record while capturing a throwaway graph (nothing runs)
    st["dec"].set_rows(st.get("row_sets"))
    g = torch.cuda.CUDAGraph()
    ops.call = rec
    try:
        with torch.cuda.graph(g):
            pipe._step(st)
    finally:
        ops.call = orig
        st["dec"].set_rows(None)
    with open(out, "w") as f:
        json.dump(descs, f)
    print(f"{len(descs)} conv launches per step recorded", flush=True)


def analyse(trace, descs_path, keys_out=None):
    descs = json.load(open(descs_path))
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # one entry per dc_conv_gemm launch: a two-kernel skinny split-K's reduce dispatch is added to its skinny kernel
    conv = []
    for r in rows:
        if "skinny_reduce_kernel" in r[2] and conv:
            s0, e0, n0 = conv[-1]
            conv[-1] = (s0, e0 + (r[1] - r[0]), n0)
        elif any(k in r[2] for k in ("conv_gemm_kernel", "conv_halo_kernel", "conv_skinny_kernel",
                                     "conv_resident_kernel")):
            conv.append(r)
    n = len(descs)
    last = conv[-n:]   # the final step of the last call is the last n conv dispatches (final decode is dense:
    # skip back over the final decode's convs by aligning on shapes below)
    # align: the final decode after the loop adds TAESD convs; find the window whose count matches the step
    best = None
    for off in range(0, min(len(conv) - n, 200) + 1):
        win = conv[len(conv) - n - off:len(conv) - off]
        fam = lambda a: ("halo" if 23 <= a <= 36 or 62 <= a <= 66 else "skinny" if 43 <= a <= 54  # noqa: E731
                         else "resident" if 55 <= a <= 58 else "gemm")
        ok = sum(fam(d["algo"]) in w[2] for w, d in zip(win, descs))
        if best is None or ok > best[0]:
            best = (ok, win)
        if ok == n:
            break
    ok, win = best
    print(f"aligned {ok}/{n} launches by kernel family")
    groups = defaultdict(lambda: [0, 0.0, 0.0, set()])
    tot = 0.0
    for (s, e, name), d in zip(win, descs):
        us = (e - s) / 1e3
        key = (d["M"], d["N"], d["K"], d["mode"], d["k"], d["stride"], d["rows"] > 0)
        g = groups[key]
        g[0] += 1
        g[1] += us
        g[2] += d["flops"]
        g[3].add((d["algo"], d["split"]))
        tot += us
    print(f"conv time in one step: {tot / 1e3:.3f} ms over {n} launches")
    if keys_out:   # per table key: launches, us in the step, the (algo, split) it ran
        per = defaultdict(lambda: [0, 0.0, None])
        for (s, e, name), d in zip(win, descs):
            if "key" in d:
                k = json.dumps(d["key"])
                per[k][0] += 1
                per[k][1] += (e - s) / 1e3
                per[k][2] = [d["algo"], d["split"]]
        with open(keys_out, "w") as f:
            json.dump(per, f, indent=0)
    for key, (cnt, us, fl, algos) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        M, N, K, mode, k, stride, rl = key
        print(f"M={M:7d}{'r' if rl else ' '} N={N:5d} K={K:6d} mode={mode} k={k} s={stride} x{cnt:3d}: {us:8.1f} us "
              f"({100 * us / tot:5.1f} %) {fl / (us * 1e-6) / 1e12:7.1f} TF/s  {sorted(algos)}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--frame", default="576,768,500,uniform",
                    help="height,width,points,pattern of the synthetic frame (C4: 352,1216,0,beams; C5 with "
                         "--batch 10: 900,1600,3000,uniform)")
    ap.add_argument("--trace")
    ap.add_argument("--descs")
    ap.add_argument("--keys-out", help="(with --trace) per-table-key step time as JSON")
    a = ap.parse_args()
    if a.trace:
        analyse(a.trace, a.descs, a.keys_out)
    else:
        h, w, n, pat = a.frame.split(",")
        record(a.out, a.batch, (int(h), int(w), int(n), pat))


if __name__ == "__main__":
    main()

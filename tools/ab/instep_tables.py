"""In-step choice of conv variants.  The tuner times each shape alone, with its caches flushed and no fused-GroupNorm
epilogue, and that misranks some shapes for the graph-replayed step (profiles/r05ag/).  Here the runners-up are
timed inside the step instead.

  make <committed.json> <top.json> <out_prefix> [n] [skip]
      Write n alternative tables (default 3).  Table i gives every shape its (skip + i)-th fastest isolated variant
      that differs from the committed choice; a shape with fewer runners-up keeps the committed choice.  A table changes
      every shape at once, so one step profile per table times one alternative for every shape.
  pick <committed.json> <out.json> <keys_committed.json> <table_1.json> <keys_1.json> [<table_2.json> <keys_2.json> ...]
      keys_*.json come from tools/step_profile.py --keys-out over each table.  Each shape takes the table whose
      launches of it ran fastest in the step, and only when that beats the committed choice by more than 3 %
      and 0.5 us per step.
"""
import json
import sys


def load(path):
    return {tuple(e["key"]): (e["algo"], e["splitk"]) for e in json.load(open(path))}


def save(table, path):
    json.dump([{"key": list(k), "algo": a, "splitk": s} for k, (a, s) in sorted(table.items())], open(path, "w"),
              indent=0)


def make(committed, top, prefix, n=3, skip=0):
    base = load(committed)
    tops = {tuple(e["key"]): [(c[0], c[1]) for c in e["top"]] for e in json.load(open(top))}
    for i in range(1, n + 1):
        t = dict(base)
        changed = 0
        for k, cands in tops.items():
            alts = [c for c in cands if c != base.get(k)]
            if k in base and len(alts) >= skip + i:
                t[k] = alts[skip + i - 1]
                changed += 1
        save(t, f"{prefix}{i}.json")
        print(f"{prefix}{i}.json: {changed} shapes on their runner-up {skip + i}")


def pick(committed, out, keys0, rest):
    base = load(committed)
    step0 = {tuple(json.loads(k)): v for k, v in json.load(open(keys0)).items()}
    arms = []
    for tp, kp in zip(rest[0::2], rest[1::2]):
        arms.append((load(tp), {tuple(json.loads(k)): v for k, v in json.load(open(kp)).items()}))
    final = dict(base)
    saved = 0.0
    for k, (cnt, us0, ran0) in sorted(step0.items()):
        best = (us0, None)
        for table, step in arms:
            if k in step and step[k][0] == cnt and table.get(k) != base.get(k) and step[k][1] < best[0]:
                best = (step[k][1], table[k])
        if best[1] is not None and best[0] < us0 * 0.97 and us0 - best[0] > 0.5 and k in base:
            final[k] = best[1]
            saved += us0 - best[0]
            print(f"{k}: {base[k]} {us0:.1f} us -> {best[1]} {best[0]:.1f} us  (x{cnt})")
    save(final, out)
    print(f"{sum(1 for k in final if final[k] != base.get(k))} shapes changed, {saved:.1f} us per step")


if __name__ == "__main__":
    if sys.argv[1] == "make":
        make(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]) if len(sys.argv) > 5 else 3,
             int(sys.argv[6]) if len(sys.argv) > 6 else 0)
    else:
        pick(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:])

"""Tables without the skinny two-kernel split-K (its skinny_reduce launch), for the in-step choice.

  make <committed.json> <out_prefix>
      alt1: every shape on a two-kernel split (splitk < 0) takes the same variant with the in-kernel last-arriver split
      of the same count (+|s|); alt2: the same variant unsplit (1); alt3: the last-arriver split of half the count.
  pick <committed.json> <out.json> <tol> <keys_committed.json> <table_1.json> <keys_1.json> [...]
      keys_*.json from tools/step_profile.py --keys-out (a launch's reduce dispatch is charged to it).  A two-kernel
      shape takes the fastest one-launch alternative when that ran within (1 + tol) x its committed in-step time: the
      in-step time leaves out the kernel boundary the reduce launch adds (~1-2 us in a graph), which the C2 A/B sees.
"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from instep_tables import load, save  # noqa: E402


SKINNY = range(43, 55)   # skinny algo ids: there splitk < 0 is the two-kernel split (elsewhere it means stream-K)


def two_kernel(v):
    return v[0] in SKINNY and v[1] < 0


def make(committed, prefix):
    base = load(committed)
    alts = [lambda s: -s, lambda s: 1, lambda s: max(1, (-s) // 2)]
    for i, f in enumerate(alts, 1):
        t = {k: ((a, f(s)) if two_kernel((a, s)) else (a, s)) for k, (a, s) in base.items()}
        save(t, f"{prefix}{i}.json")
        print(f"{prefix}{i}.json: {sum(1 for k in base if two_kernel(base[k]))} two-kernel shapes changed")


def pick(committed, out, tol, keys0, rest):
    base = load(committed)
    step0 = {tuple(json.loads(k)): v for k, v in json.load(open(keys0)).items()}
    arms = [(load(tp), {tuple(json.loads(k)): v for k, v in json.load(open(kp)).items()})
            for tp, kp in zip(rest[0::2], rest[1::2])]
    final = dict(base)
    delta = 0.0
    for k, (cnt, us0, ran0) in sorted(step0.items()):
        if k not in base or not two_kernel(base[k]):
            continue
        best = (float("inf"), None)
        for table, step in arms:
            if k in step and step[k][0] == cnt and step[k][1] < best[0]:
                best = (step[k][1], table[k])
        if best[1] is not None and best[0] <= us0 * (1 + tol):
            final[k] = best[1]
            delta += best[0] - us0
            print(f"{k}: {base[k]} {us0:.1f} us -> {best[1]} {best[0]:.1f} us  (x{cnt})")
        else:
            print(f"{k}: {base[k]} {us0:.1f} us kept (best one-launch {best[1]} {best[0]:.1f} us)")
    save(final, out)
    n = sum(1 for k in final if final[k] != base.get(k))
    print(f"{n} shapes changed, {delta:+.1f} us per step of busy time")


if __name__ == "__main__":
    if sys.argv[1] == "make":
        make(sys.argv[2], sys.argv[3])
    else:
        pick(sys.argv[2], sys.argv[3], float(sys.argv[4]), sys.argv[5], sys.argv[6:])

"""Keep from a --try re-tune only the level-0/1-style skinny swaps the C2 step profile confirmed (profiles/r05ag/):
3x3 shapes with ktot >= 5760 moving to a skinny variant; every other shape keeps the committed entry.
Usage: python tools/ab/filter_table.py <committed.json> <retuned.json> <out.json>"""
import json
import sys

old = {tuple(e["key"]): (e["algo"], e["splitk"]) for e in json.load(open(sys.argv[1]))}
new = json.load(open(sys.argv[2]))
n = 0
for e in new:
    k = tuple(e["key"])
    take = k[8] == 3 and k[11] >= 5760 and 43 <= e["algo"] <= 54
    if k in old and not take:
        e["algo"], e["splitk"] = old[k]
    elif k in old and (e["algo"], e["splitk"]) != old[k]:
        n += 1
        print(k, old[k], "->", (e["algo"], e["splitk"]))
json.dump(new, open(sys.argv[3], "w"), indent=0)
print(n, "entries changed")

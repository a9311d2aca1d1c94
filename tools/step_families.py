import csv, re, sys
from collections import defaultdict
def fam(n):
    n=n.replace("(anonymous namespace)::","")
    for k in ("conv_gemm_kernel","conv_halo_kernel","conv_skinny_kernel","skinny_reduce","conv_resident_kernel","attn_fwd","attn_bwd_dq","attn_bwd_dkdv","gn_","ln_","cross_mfma","upsample","memset"):
        if k in n: return k
    return re.sub(r"[<(].*","",n)[:40]
rows=[]
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),r["Kernel_Name"]))
rows.sort()
# last step: find last attn_fwd L0 ... simpler: take the last N kernels where N = kernels per step
N=int(sys.argv[2])
# find window: step = sequence between consecutive occurrences of first kernel?  use last 3N and take the middle N
win=rows[-2*N:-N] if len(rows)>=2*N else rows[-N:]
agg=defaultdict(lambda:[0,0.0])
for s,e,n in win:
    f=fam(n); agg[f][0]+=1; agg[f][1]+=(e-s)/1e3
tot=sum(v[1] for v in agg.values())
print(f"window {len(win)} kernels, busy {tot/1e3:.3f} ms, wall {(win[-1][1]-win[0][0])/1e6:.3f} ms")
for k,(c,t) in sorted(agg.items(), key=lambda kv:-kv[1][1]): print(f"{k:30s} x{c:4d} {t:9.1f} us {100*t/tot:5.1f}%")
# optional third argument "names": the same window per kernel name (template arguments kept)
if len(sys.argv) > 3 and sys.argv[3] == "names":
    byname = defaultdict(lambda: [0, 0.0])
    for s, e, n in win:
        k = n.replace("(anonymous namespace)::", "").replace("void ", "")
        k = re.sub(r"\(.*", "", k)[:70]
        byname[k][0] += 1
        byname[k][1] += (e - s) / 1e3
    print("-- per kernel name")
    for k, (c, t) in sorted(byname.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:70s} x{c:4d} {t:9.1f} us")

"""Steady-state busy picture of a rocprofv3 kernel trace of the pipelined bench:
per kernel family the mean duration and the share of the span during which at least
one instance runs, and what runs while no expansion does."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
rows.sort(key=lambda r: r["s"])
exp = [r for r in rows if r["k"] == "expand_kernel"]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 4     # warm-up expansions (and the alone batch at the end)
t0, t1 = exp[skip]["s"], exp[-2]["s"]
nb = len(exp) - 2 - skip
win = [r for r in rows if r["e"] > t0 and r["s"] < t1]


def union(iv):
    iv = sorted((max(s, t0), min(e, t1)) for s, e in iv if e > t0 and s < t1)
    tot, cs, ce = 0, None, None
    out = []
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                out.append((cs, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        out.append((cs, ce))
    return out


span = t1 - t0
print(f"span {span / 1e3:.1f} us over {nb} batches: {span / 1e3 / nb:.1f} us per batch")
fam = defaultdict(list)
for r in win:
    fam[r["k"]].append(r)
for k, rs in sorted(fam.items(), key=lambda kv: -sum(r["e"] - r["s"] for r in kv[1])):
    u = union([(r["s"], r["e"]) for r in rs])
    cov = sum(e - s for s, e in u)
    print(f"{k[:26]:26s} n {len(rs):4d} mean {sum(r['e'] - r['s'] for r in rs) / len(rs) / 1e3:8.1f} us  busy {cov / span:6.1%}")
ue = union([(r["s"], r["e"]) for r in exp])
gaps = []
prev = t0
for s, e in ue:
    if s > prev:
        gaps.append((prev, s))
    prev = e
if prev < t1:
    gaps.append((prev, t1))
idle = defaultdict(float)
for gs, ge in gaps:
    for r in win:
        o = min(r["e"], ge) - max(r["s"], gs)
        if o > 0 and r["k"] != "expand_kernel":
            idle[r["k"]] += o / 1e3
g = sum(e - s for s, e in gaps)
print(f"no expansion running: {g / 1e3 / nb:.1f} us per batch; kernels then (us per batch):",
      {k: round(v / nb, 1) for k, v in idle.items()})

"""Summarise a rocprofv3 kernel trace of the pipelined bench: per expansion launch its
duration and the gap before it (expansion-stream idle), plus what ran in the gaps."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
rows.sort(key=lambda r: r["s"])
exp = [r for r in rows if r["k"].startswith("expand_kernel")]
print("expansions", len(exp))
gaps = []
for a, b in zip(exp, exp[1:]):
    gap = b["s"] - a["e"]
    inside = defaultdict(float)
    for r in rows:
        if r["e"] > a["e"] and r["s"] < b["s"] and not r["k"].startswith("expand"):
            inside[r["k"][:28]] += (min(r["e"], b["s"]) - max(r["s"], a["e"])) / 1e3
    gaps.append(gap)
    print(f"exp {(a['e'] - a['s']) / 1e3:8.1f} us  gap {gap / 1e3:7.1f} us  ", {k: round(v, 1) for k, v in inside.items()})
span = (exp[-1]["e"] - exp[0]["s"]) / 1e3
print(f"span {span:.1f} us over {len(exp)} expansions: {span / len(exp):.1f} us each; mean gap {sum(gaps) / max(1, len(gaps)) / 1e3:.1f} us")

"""Steady-state timeline of the pipelined C2 bench from a rocprofv3 kernel trace:
the expansion stream's gaps (end of one expansion to the start of the next) and
what ran in them, the per-kernel busy time per batch, and the walks' spans.
usage: python scripts/timeline.py kernel_trace.csv [skip_batches]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 4
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
rows.sort(key=lambda r: r["s"])
exps = [r for r in rows if r["k"] == "expand_kernel"]
exps = exps[skip:-2] if len(exps) > skip + 4 else exps
t0, t1 = exps[0]["s"], exps[-1]["e"]
win = [r for r in rows if r["e"] > t0 and r["s"] < t1]
nb = len(exps)
print(f"{nb} expansions, {(t1 - t0) / 1e3 / nb:.1f} us per batch (start of first to end of last / count)")
print("expansion durations (us):", " ".join(f"{(x['e'] - x['s']) / 1e3:.0f}" for x in exps))
gaps = []
for a, b in zip(exps, exps[1:]):
    g = (b["s"] - a["e"]) / 1e3
    during = [r for r in win if r["s"] < b["s"] and r["e"] > a["e"] and r["k"] != "expand_kernel"]
    gaps.append(g)
    names = collections.Counter(r["k"] for r in during)
    print(f"gap {g:7.1f} us  running: " + ", ".join(f"{k} x{v}" for k, v in names.most_common()))
print(f"mean gap {sum(gaps) / max(1, len(gaps)):.1f} us")
busy = collections.defaultdict(float)
for r in win:
    busy[r["k"]] += (min(r["e"], t1) - max(r["s"], t0)) / 1e3
print("kernel time inside the window, per batch (us):")
for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v / nb:9.1f}")
walks = [r for r in win if r["k"] == "segments_kernel"]
print("walks (start rel, dur us):", " ".join(f"{(w['s'] - t0) / 1e3:.0f}/{(w['e'] - w['s']) / 1e3:.0f}" for w in walks))

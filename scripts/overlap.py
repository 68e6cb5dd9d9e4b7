"""Concurrency in a kernel trace of the pipelined bench: for each segment walk and
expansion, its duration and the time it shared the GPU with walks / expansions."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
rows.sort(key=lambda r: r["s"])
t0 = rows[0]["s"]
big = [r for r in rows if r["k"] in ("segments_kernel", "expand_kernel")]


def ov(a, b):
    return max(0, min(a["e"], b["e"]) - max(a["s"], b["s"])) / 1e3


for r in big:
    w = sum(ov(r, o) for o in big if o is not r and o["k"] == "segments_kernel")
    x = sum(ov(r, o) for o in big if o is not r and o["k"] == "expand_kernel")
    print(f"{r['k'][:8]} start {(r['s'] - t0) / 1e3:9.1f} dur {(r['e'] - r['s']) / 1e3:7.1f} us  with walks {w:7.1f}  with expansions {x:7.1f}")

"""Walk-stream gaps in a rocprofv3 kernel trace of the pipelined C2 bench: for each
segment walk, the idle time since the previous walk ended and the end of the last
small (construction / draws) kernel before it started."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
rows.sort(key=lambda r: r["s"])
t0 = rows[0]["s"]
walks = [r for r in rows if r["k"] == "segments_kernel"]
exps = [r for r in rows if r["k"] == "expand_kernel"]
small = [r for r in rows if r["k"] not in ("segments_kernel", "expand_kernel")]
prev = None
for w in walks:
    before = [r for r in small if r["e"] <= w["s"]]
    last = max(before, key=lambda r: r["e"]) if before else None
    gap = (w["s"] - prev["e"]) / 1e3 if prev else 0
    lag = (w["s"] - last["e"]) / 1e3 if last else 0
    ex = sum(max(0, min(w["e"], x["e"]) - max(w["s"], x["s"])) for x in exps) / 1e3
    print(f"walk start {(w['s'] - t0) / 1e3:9.1f} dur {(w['e'] - w['s']) / 1e3:7.1f} gap {gap:6.1f} us; last small kernel "
          f"{last['k'] if last else '-':22s} ended {lag:6.1f} us before; with expansions {ex:7.1f} us")
    prev = w
for k in sorted(set(r["k"] for r in small)):
    d = [(r["e"] - r["s"]) / 1e3 for r in small if r["k"] == k]
    print(f"{k:24s} n={len(d):3d} mean {sum(d) / len(d):8.1f} us max {max(d):8.1f}")

"""Print per-kernel mean durations from a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)]:
    name = r["Name"]
    short = name.split("(")[0] if not name.startswith("void") else name.split("(")[1].split(")")[-1] if False else name
    short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{short[:40]:40s} calls={r['Calls']:>3s} avg={float(r['AverageNs'])/1e3:9.1f} us  {float(r['Percentage']):5.1f} %")

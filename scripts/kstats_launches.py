"""Per-launch-shape mean durations of one kernel from a rocprofv3 kernel_trace.csv.

The gated C2 schedule runs the first batch of each run as two half-day windows
(PipelineConfig.first_split), so rocprofv3's per-kernel mean mixes full-day and
half-day expansion launches; this groups the launches by grid shape.
usage: python scripts/kstats_launches.py kernel_trace.csv [KERNEL_SUBSTRING]"""
import collections
import csv
import sys

want = sys.argv[2] if len(sys.argv) > 2 else "expand_kernel"
groups = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if want not in r["Kernel_Name"]:
        continue
    wg = int(r["Workgroup_Size_X"]) or 1
    shape = (int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    groups[shape].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(len(v) for v in groups.values())
for shape, v in sorted(groups.items(), key=lambda kv: -len(kv[1])):
    print(f"{want} grid {shape[0]}x{shape[1]}x{shape[2]} workgroups: calls={len(v):3d} avg={sum(v) / len(v):9.1f} us"
          f"  ({len(v)} of {tot} launches)")

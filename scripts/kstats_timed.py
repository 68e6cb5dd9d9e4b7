"""Mean duration of the dominant kernel over the timed steps of one bench run, from a
rocprofv3 kernel trace: the launches of KERNEL in start order, the last one being bench.py's
`alone` batch, the STEPS before it the timed region's (pre-warm and warm-up launches come first).
usage: python scripts/kstats_timed.py kernel_trace.csv STEPS [KERNEL]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
name = sys.argv[3] if len(sys.argv) > 3 else "expand_kernel"
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if name in r["Kernel_Name"])
timed, alone = ks[-steps - 1:-1], ks[-1]
d = [(e - s) / 1e3 for s, e in timed]
print(f"{name}: {len(ks)} launches; the {steps} timed: mean {sum(d) / len(d):.1f} us "
      f"(min {min(d):.1f}, max {max(d):.1f}); the alone launch {(alone[1] - alone[0]) / 1e3:.1f} us")

"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh) per kernel: mean per dispatch.
FETCH_SIZE/WRITE_SIZE are in KB (rocprofv3 derived counters); on gfx950 FETCH_SIZE
reads half the bytes of wide streaming loads (MI355X_MICROARCH.md, HBM)."""
import collections
import csv
import glob
import re
import sys

KERNELS = ["expand_kernel<float>", "expand_kernel<double>", "segments_kernel", "minute_draws_kernel",
           "init_kernel", "geom_kernel", "event_draws_kernel", "events_kernel", "desc_kernel", "commit_kernel",
           "chain_kernel"]


def key(name):
    for k in KERNELS:
        if k.split("<")[0] in name and (("<" not in k) or k.split("<")[1][:-1] in name):
            return k
    return None


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(f"{d}/p*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = key(r["Kernel_Name"])
            if k:
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    out = {}
    for k, d2 in agg.items():
        out[k] = {c: v / len(disp[k][c]) for c, v in d2.items()}
        print(k)
        print("   " + ", ".join(f"{c}={v:.4g}" for c, v in sorted(out[k].items())))
    return out


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh) per kernel: mean per dispatch.
FETCH_SIZE/WRITE_SIZE are in KB (rocprofv3 derived counters); on gfx950 FETCH_SIZE
reads half the bytes of wide streaming loads (MI355X_MICROARCH.md, HBM)."""
import collections
import csv
import glob
import re
import sys

KERNELS = ["expand_kernel<float>", "expand_kernel<double>", "segments_kernel", "minute_table_kernel", "fixup_kernel",
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


def write_traffic(d, chains, seconds, precision="fp32", mode="trace", kernel="expand_kernel<float>", out=None):
    """profiles/pmc_traffic.json: HBM bytes per launch of the bench's dominant kernel.
    FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is doubled (gfx950 reports half the
    bytes of wide streaming reads, MI355X_MICROARCH.md § HBM)."""
    import json
    import os
    s = main(d)[kernel]
    fetch = s["FETCH_SIZE"] * 1024 * 2
    write = s["WRITE_SIZE"] * 1024
    rec = {"kernel": kernel, "chains": chains, "seconds": seconds, "precision": precision, "mode": mode,
           "fetch_bytes_corrected": fetch, "fetch_size_kib_raw": s["FETCH_SIZE"], "write_bytes": write,
           "traffic_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": 12 * chains * seconds,
           "source": os.path.basename(os.path.normpath(d))}
    out = out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                              "pmc_traffic.json")
    json.dump(rec, open(out, "w"), indent=1)
    return rec

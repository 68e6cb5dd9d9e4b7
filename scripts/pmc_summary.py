"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh, scripts/pmc_workload.sh) per
kernel: mean per dispatch.  FETCH_SIZE/WRITE_SIZE are in KiB (rocprofv3 derived
counters); on gfx950 FETCH_SIZE reads half the bytes of wide streaming loads
(MI355X_MICROARCH.md, HBM), so it is doubled before it is called traffic.

  python3 scripts/pmc_summary.py DIR                  print the per-kernel means
  python3 scripts/pmc_summary.py DIR --record K=V ... upsert the dominant expand
        kernel's record into profiles/pmc_kernels.json (keys: workload, chains,
        launch_seconds, precision, mode, cc), which bench.py reads
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """'void (anonymous namespace)::expand_kernel<float, 1, false>(...)' -> 'expand_kernel<float, 1, false>'"""
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("tmh::", "")
    depth, out = 0, []
    for ch in n:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return re.sub(r"\s+", " ", "".join(out)).strip()


def main(d, quiet=False):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(f"{d}/p*/*counter_collection.csv") + glob.glob(f"{d}/p*/*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    out = {}
    for k, d2 in sorted(agg.items()):
        out[k] = {c: v / len(disp[k][c]) for c, v in d2.items()}
        out[k]["_dispatches"] = max(len(s) for s in disp[k].values())
        if not quiet:
            print(k)
            print("   " + ", ".join(f"{c}={v:.4g}" for c, v in sorted(out[k].items())))
    return out


def record(d, **key):
    """profiles/pmc_kernels.json: the expand kernel's per-launch counters on one workload."""
    s = main(d, quiet=True)
    exp = [k for k in s if k.startswith("expand_kernel<")]
    if not exp:
        raise SystemExit(f"no expand_kernel dispatch in {d}")
    k = max(exp, key=lambda k: s[k].get("SQ_WAVES", 0) * s[k]["_dispatches"])
    c = s[k]
    rec = dict(key)
    sys.path.insert(0, ROOT)
    from tmhpvsim_amd.build import build_stamp
    rec.update(kernel=k, dispatches=c["_dispatches"], source=os.path.basename(os.path.normpath(d)),
               build_stamp=build_stamp())   # bench.py ignores a record of another build
    for name, cn in (("valu_insts_per_launch", "SQ_INSTS_VALU"), ("salu_insts_per_launch", "SQ_INSTS_SALU"),
                     ("trans_f32_insts_per_launch", "SQ_INSTS_VALU_TRANS_F32"), ("waves_per_launch", "SQ_WAVES"),
                     ("wave_cycles", "SQ_WAVE_CYCLES"), ("wait_any", "SQ_WAIT_ANY"),
                     ("wait_inst_any", "SQ_WAIT_INST_ANY"), ("active_inst_any", "SQ_ACTIVE_INST_ANY"),
                     ("active_inst_valu", "SQ_ACTIVE_INST_VALU")):
        if cn in c:
            rec[name] = c[cn]
    mix = {cn[len("SQ_INSTS_VALU_"):]: c[cn] for cn in sorted(c) if cn.startswith("SQ_INSTS_VALU_")}
    if len(mix) > 1:   # per-type VALU wave-instructions (bench.py weighs them by issue cycles)
        rec["valu_mix"] = mix
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rec["fetch_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
        rec["write_bytes"] = c["WRITE_SIZE"] * 1024
        rec["traffic_bytes_per_launch"] = rec["fetch_bytes_corrected"] + rec["write_bytes"]
    path = os.path.join(ROOT, "profiles", "pmc_kernels.json")
    try:
        db = json.load(open(path))
    except (OSError, ValueError):
        db = {"note": "per-launch PMC means of the dominant expand kernel per bench workload "
                      "(scripts/pmc_workload.sh); SQ_* are wave-instruction counts summed over the chip",
              "records": []}
    ident = ("workload", "chains", "launch_seconds", "precision", "mode", "cc", "compact")
    db["records"] = [r for r in db["records"] if any(r.get(i) != rec.get(i) for i in ident)] + [rec]
    json.dump(db, open(path, "w"), indent=1)
    return rec


def _val(v):
    try:
        return int(v)
    except ValueError:
        return v


if __name__ == "__main__":
    if "--record" in sys.argv:
        i = sys.argv.index("--record")
        kv = dict(a.split("=", 1) for a in sys.argv[i + 1:])
        print(json.dumps(record(sys.argv[1], **{k: _val(v) for k, v in kv.items()}), indent=1))
    else:
        main(sys.argv[1])

#!/bin/bash
# One C2 bench with the --timeline diagnostic; prints the expansion stream's gaps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timeline "$@" > gpurun_out/tl.json 2> gpurun_out/tl.err || { tail -5 gpurun_out/tl.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/tl.json").read())
t = d["timeline"]
f = lambda v: " ".join(f"{x:.3f}" for x in v)
print("ms/step %.3f expand %.3f" % (d["ms_per_step"], d["roofline"]["kernel_ms"]))
for k, v in t.items():
    print(f"{k:34s} mean {sum(v) / max(1, len(v)):.3f}: {f(v)}")
PY

#!/bin/bash
# Same-box A/B of whole source trees (each a `git archive` of one revision under _ab/REV with its
# own built library), alternating the trees so box drift hits all of them alike:
#   bash scripts/tree_ab.sh TAG REPS 'name|tree dir (. = this tree)|bench args' ...
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1 REPS=$2; shift 2
for rep in $(seq 1 "$REPS"); do
  for spec in "$@"; do
    IFS='|' read -r name dir args <<< "$spec"
    out=$ROOT/gpurun_out/tab_${TAG}_${name}_$rep
    (cd "$dir" && timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none $args > "$out.json" 2> "$out.err") \
      || { echo "$name failed rc=$?"; tail -3 "$out.err"; exit 1; }
    python3 - "$out.json" "$name" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d.get("roofline") or {}
al = (r.get("alone") or {}).get("kernel_ms")
print("%-10s value %.4g ms/step %.3f expand %.3f alone %s" % (sys.argv[2], d["value"], d["ms_per_step"], r.get("kernel_ms") or 0, al),
      {k: round(v, 3) for k, v in (d.get("phases_ms") or {}).items() if v})
EOF
  done
done

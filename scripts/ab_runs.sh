#!/bin/bash
# One bench line per named run (current library unless LIB is given), printed compactly:
#   bash scripts/ab_runs.sh TAG 'name|lib|bench args' ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for spec in "$@"; do
  IFS='|' read -r name lib args <<< "$spec"
  l=$PWD/tmhpvsim_amd/libtmhpvsim.so; [ "$lib" = cur ] || l=$PWD/tmhpvsim_amd/libtmh_$lib.so
  TMHPVSIM_LIB=$l timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none $args \
      > gpurun_out/ab_${TAG}_$name.json 2> gpurun_out/ab_${TAG}_$name.err || { echo "$name failed rc=$?"; tail -3 gpurun_out/ab_${TAG}_$name.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_${TAG}_$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', 'value %.4g ms/step %.2f kernel %.3f alone %s' % (d['value'], d['ms_per_step'], r.get('kernel_ms') or 0, (r.get('alone') or {}).get('kernel_ms')), d.get('projected_node_value'))"
done

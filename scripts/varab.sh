#!/bin/bash
# Same-box A/B of (library, bench arguments) variants: varab.sh TAG 'name|lib|args' ...
# lib "cur" = libtmhpvsim.so, else tmhpvsim_amd/libtmh_<lib>.so
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="$1"; shift
for rep in 1 2; do
for spec in "$@"; do
  IFS='|' read -r name lib bargs <<< "$spec"
  so=$PWD/tmhpvsim_amd/libtmh_$lib.so; [ "$lib" = cur ] && so=$PWD/tmhpvsim_amd/libtmhpvsim.so
  TMHPVSIM_LIB=$so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $bargs > gpurun_out/vab_${TAG}_$name.json 2> gpurun_out/vab_${TAG}_$name.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/vab_${TAG}_$name.json').read()); r=d['roofline']
print('$name value %.4g ms/step %.3f expand %.3f alone %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], (r.get('alone') or {}).get('kernel_ms', float('nan'))), {k: round(v, 3) for k, v in d['phases_ms'].items() if v})"
done
done

#!/bin/bash
# Same-box A/B of library builds: libab.sh TAG variant... ("cur" = libtmhpvsim.so, else libtmh_<v>.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="$1"; shift
for rep in 1 2; do
for v in "$@"; do
  lib=$PWD/tmhpvsim_amd/libtmh_$v.so; [ "$v" = cur ] && lib=$PWD/tmhpvsim_amd/libtmhpvsim.so
  b=bench.py
  TMHPVSIM_LIB=$lib timeout -k 10 300 python $b --steps 10 --warmup 3 --no-cpu-baseline ${BARGS:-} > gpurun_out/lab_${TAG}_$v.json 2> gpurun_out/lab_${TAG}_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/lab_${TAG}_$v.json').read()); r=d['roofline']
print('$v value %.4g ms/step %.3f expand %.3f alone %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['alone']['kernel_ms']), {k: round(v, 3) for k, v in d['phases_ms'].items() if v})"
done
done

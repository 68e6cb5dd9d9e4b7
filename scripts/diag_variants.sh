#!/bin/bash
# Cost breakdown of the per-second body (diagnostic builds; never the product):
# build libtmh_<variant>.so with one piece disabled each, then time the kernels.
# Build here:  bash scripts/diag_variants.sh build ;  run on the GPU box:  bash scripts/diag_variants.sh run
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
VARIANTS="${VARIANTS:-base:- norng:-DTMH_DIAG_NO_RNG nondtri:-DTMH_DIAG_NO_NDTRI nopv:-DTMH_DIAG_NO_PV nostore:-DTMH_DIAG_NO_STORE}"
if [ "${1:-run}" = build ]; then
  for v in $VARIANTS; do
    name=${v%%:*}; flag=${v#*:}; [ "$flag" = "-" ] && flag=""; flag=${flag//+/ }
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off $flag \
      -I include -o tmhpvsim_amd/libtmh_$name.so tmhpvsim_amd/csrc/tmh_engine.hip || exit 1
  done
  exit 0
fi
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/diag"
mkdir -p "$OUT"
for v in $VARIANTS; do
  name=${v%%:*}
  echo "== $name"
  ( cd /tmp && TMHPVSIM_LIB=$ROOT/tmhpvsim_amd/libtmh_$name.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$OUT/$name" -o run -- python "$ROOT/bench.py" --steps ${STEPS:-3} --warmup 1 --pipeline ${PIPELINE:-1} --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$OUT/$name.json" 2> "$OUT/$name.err" ) || exit $?
  cat "$OUT/$name.json"
done

#!/bin/bash
# Walk-alone and C2 bench A/B of library builds: walk_ab.sh TAG variant... ("cur" = libtmhpvsim.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
for v in "$@"; do
  lib=$PWD/tmhpvsim_amd/libtmh_$v.so; [ "$v" = cur ] && lib=$PWD/tmhpvsim_amd/libtmhpvsim.so
  echo "== $v"; TMHPVSIM_LIB=$lib timeout -k 10 100 python scripts/walk_only.py --reps 5 ${WARGS:-} || exit $?
done
bash scripts/libab.sh $TAG "$@"

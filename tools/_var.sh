#!/bin/bash
# GPU step: run a python tool against every variants/lib_*.so (ACTH_LIB), one process each, twice (interleaved).
# usage: tools/_var.sh <tag> <tool.py> [args]
OUT=gpurun_out/${1:-var}; TOOL=$2; shift 2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for f in variants/lib_*.so; do
    echo "== $f (rep $rep)" >> $OUT/var.log
    ACTH_LIB=$PWD/$f timeout -k 10 120 python -u $TOOL "$@" >> $OUT/var.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/var.log

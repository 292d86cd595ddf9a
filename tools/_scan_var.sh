#!/bin/bash
# GPU step: tools/bench_scan.py --quad [--shape ...] against every variants/lib_*.so (ACTH_LIB), one process each.
OUT=gpurun_out/${1:-scanvar}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in variants/lib_*.so; do
  echo "== $f" >> $OUT/var.log
  ACTH_LIB=$PWD/$f timeout -k 10 120 python -u tools/bench_scan.py --quad "$@" >> $OUT/var.log 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/var.log

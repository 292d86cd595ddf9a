#!/bin/bash
# GPU step: GEMM / conv parity tests + bench_gemm on the given SHAPES indices for every variants/lib_*.so.
# usage: tools/_gemm_var.sh <tag> <only-indices> <pytest -k expr>
OUT=gpurun_out/${1:-gvar}; ONLY=$2; KEXPR=${3:-gemm or conv}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in variants/lib_*.so; do
  echo "== $f" >> $OUT/g.log
  ACTH_LIB=$PWD/$f timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_full_geometry_gpu.py -k "$KEXPR" >> $OUT/g.log 2>&1 || exit $?
done
for rep in 1 2; do for f in variants/lib_*.so; do
  echo "== $f (rep $rep)" >> $OUT/g.log
  ACTH_LIB=$PWD/$f timeout -k 10 200 python -u tools/bench_gemm.py --tiles 0 --only $ONLY >> $OUT/g.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/g.log | grep -vE "^\s*$"

#!/bin/bash
# GPU step: flash-attention parity tests + micro-benchmark for every variants/lib_*.so (ACTH_LIB).
OUT=gpurun_out/${1:-favar}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in variants/lib_*.so; do
  echo "== $f" >> $OUT/fa.log
  ACTH_LIB=$PWD/$f timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_full_geometry_gpu.py -k "flash or ip_attn or xattn" >> $OUT/fa.log 2>&1 || exit $?
done
for rep in 1 2; do for f in variants/lib_*.so; do
  echo "== $f (rep $rep)" >> $OUT/fa.log
  ACTH_LIB=$PWD/$f timeout -k 10 120 python -u tools/bench_attn.py --flash >> $OUT/fa.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/fa.log | grep -E "==|passed|failed|flash_attn"

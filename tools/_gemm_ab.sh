#!/bin/bash
# GPU step: GEMM / model tests with the in-tree library, then bench A (in-tree) vs B (variants/lib_a_old.so).
OUT=gpurun_out/${1:-gab}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_full_geometry_gpu.py -x -v --timeout 200 \
  --timeout-method thread -k "gemm or conv or geglu or linear or orow or unet" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/_ab.sh ${OUT#gpurun_out/} "ACTH_X=0" "ACTH_LIB=$PWD/variants/lib_a_old.so" "$@"

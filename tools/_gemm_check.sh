#!/bin/bash
# GPU step: GEMM / conv / FFN kernel tests, then tools/bench_gemm.py against every variants/lib_*.so.
OUT=gpurun_out/${1:-gemm}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "gemm or conv or geglu or temporal_gemm or linear or orow" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/_var.sh ${OUT#gpurun_out/}/var tools/bench_gemm.py "$@"

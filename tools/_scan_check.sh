#!/bin/bash
# GPU step: scan tests (kernels, level shapes, SS2D goldens / model), then tools/bench_scan.py.
OUT=gpurun_out/${1:-scan}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_full_geometry_gpu.py tests/test_model_gpu.py \
  -x -v --timeout 200 --timeout-method thread -k "scan or ss2d or mamba or SS2D" > $OUT/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_scan.py > $OUT/bench_scan.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; cat $OUT/bench_scan.log; exit $rc

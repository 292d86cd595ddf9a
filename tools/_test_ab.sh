#!/bin/bash
# GPU step: selected GPU tests, then the tools/_ab.sh A/B bench + kernel trace.
# usage: tools/_test_ab.sh <tag> "<pytest -k expr>" "<envA>" "<envB>" [bench args]
TAG=$1; K=$2; EA=$3; EB=$4; shift 4
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_full_geometry_gpu.py \
  -x -v --timeout 200 --timeout-method thread -k "$K" > gpurun_out/$TAG/pytest.log 2>&1 &&
bash tools/_ab.sh $TAG "$EA" "$EB" "$@"
rc=$?; tail -4 gpurun_out/$TAG/pytest.log; exit $rc

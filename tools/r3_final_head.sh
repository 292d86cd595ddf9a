#!/bin/bash
# Final round-3 GPU pass at HEAD: gpu tests + smoke + bench + 3-branch kernel trace (gpu_check.sh), then a
# separate kernel trace of the mode-2 (4-branch, C4 = C5's per-rank workload) step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3head}
bash tools/gpu_check.sh $TAG || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_m2 -o run -- python3 -u bench.py --mode 2 \
    --steps 2 --warmup 1 --no-cpu-baseline --no-four-branch-compare --no-other-modes > gpurun_out/$TAG/prof_m2.log 2>&1

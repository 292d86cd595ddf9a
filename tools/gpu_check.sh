#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench line, rocprofv3 kernel stats. Every GPU step is
# time-limited and the chain stops at the first failure. Usage: tools/gpu_check.sh <tag> [bench args]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ACTH_PARITY_LOG=$PWD/$OUT/parity.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 400 python -u bench.py "$@" > "$OUT/bench.log" 2>&1 &&
ACTH_TRACE_MARK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 -u bench.py \
    --steps 4 --warmup 1 --no-cpu-baseline --no-four-branch-compare --no-other-modes --no-fp16-compare --no-fpb25 \
    > "$OUT/prof.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"; tail -2 "$OUT/smoke.log"; tail -1 "$OUT/bench.log"
exit $rc

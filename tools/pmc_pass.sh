#!/bin/bash
# HBM traffic counters for one short bench run: FETCH_SIZE and WRITE_SIZE in separate passes
# (they do not fit one pass on gfx950). Usage: tools/pmc_pass.sh <outdir> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ACTH_WORKLOAD_OUT="$OUT/workload.txt"     # bench.py writes the counted run's workload key
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -f csv -d "$OUT/$C" -o run -- \
      python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --no-four-branch-compare --no-other-modes --no-fp16-compare --no-fpb25 "$@" > "$OUT/$C.log" 2>&1 || exit $?
done

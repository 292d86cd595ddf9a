#!/bin/bash
# Evidence at HEAD for the round's profiles/. Part A: PMC traffic passes (FETCH_SIZE / WRITE_SIZE) ->
# profiles/pmc_traffic.json (read by the bench line's traffic fields), then gpu tests, smoke, the default bench
# line and a marked kernel trace (tools/gpu_check.sh). Part B: the mode-2 kernel trace and the C1-geometry bench.
# Usage: tools/head_evidence.sh <tag> <A|B> <round> <sha>
set -o pipefail
TAG=${1:-head}; PART=${2:-A}; ROUND=${3:-r5}; SHA=${4:-HEAD}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$PART" = A ]; then
  bash tools/pmc_pass.sh "$OUT/pmc" || exit $?
  python tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_traffic.csv" || exit $?
  python tools/pmc_summary.py "$OUT/pmc" --json profiles/pmc_traffic.json --workload "$(cat "$OUT/pmc/workload.txt")" \
      --source "profiles/${ROUND}_pmc_traffic.csv (tools/pmc_pass.sh: bench.py --steps 1 --warmup 0, mode 0 default config, FETCH_SIZE and WRITE_SIZE passes, $ROUND HEAD $SHA)" || exit $?
  cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
  bash tools/gpu_check.sh "$TAG"
  exit $?
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_m2" -o run -- python3 -u bench.py --mode 2 \
    --steps 2 --warmup 1 --no-cpu-baseline --no-four-branch-compare --no-other-modes --no-fp16-compare --no-fpb25 \
    > "$OUT/prof_m2.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --width 576 --no-cpu-baseline --no-other-modes --no-fp16-compare --no-fpb25 \
    > "$OUT/bench_C1_576x576.log" 2>&1
rc=$?
tail -1 "$OUT/bench_C1_576x576.log"
exit $rc

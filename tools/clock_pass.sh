#!/bin/bash
# Effective shader clock per kernel (MI355X_MICROARCH.md, DVFS: GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time) for
# one short bench run per activation dtype. Usage: tools/clock_pass.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/clock}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for DT in bf16 fp16; do
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$OUT/$DT" -o run -- \
      python3 -u bench.py --steps 2 --warmup 1 --dtype $DT --no-cpu-baseline --no-roofline --no-four-branch-compare \
      --no-other-modes > "$OUT/$DT.log" 2>&1 || exit $?
done
python3 tools/clock_summary.py "$OUT/bf16" "$OUT/fp16"

#!/bin/bash
# Round-end evidence for bench.py's default command: a rocprofv3 kernel trace with per-kernel stats
# (one timed run) and the two HBM-traffic PMC passes (tools/pmc_pass.sh, one sampler step each).
# Usage: tools/profile_head.sh <outdir>; then on the CPU side:
#   python tools/pmc_summary.py <outdir>/pmc --json profiles/pmc_traffic.json --source <tag>
set -o pipefail
OUT=${1:-gpurun_out/prof_head}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-four-branch-compare > "$OUT/trace.log" 2>&1 || exit $?
bash tools/pmc_pass.sh "$OUT/pmc"

#!/bin/bash
# A/B: bench.py with env A vs env B (same box, back to back), then a kernel-trace of A.
# usage: tools/_ab.sh <tag> "<envA>" "<envB>" [bench args]
TAG=$1; EA=$2; EB=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
env $EA timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-four-branch-compare --no-other-modes "$@" > $OUT/bench_a.log 2>&1 &&
env $EB timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-four-branch-compare --no-other-modes "$@" > $OUT/bench_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-four-branch-compare --no-other-modes --no-roofline "$@" > $OUT/prof.log 2>&1
rc=$?
for f in a b; do python - $OUT/bench_$f.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'], (d.get('roofline') or {}).get('frac'))
PY
done
exit $rc

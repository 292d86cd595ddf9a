#!/bin/bash
# GPU step: bench.py against every variants/lib_*.so, interleaved twice (same box), then ms/step per variant.
OUT=gpurun_out/${1:-ab3}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do for f in variants/lib_*.so; do
  n=$(basename $f .so)
  ACTH_LIB=$PWD/$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-four-branch-compare --no-other-modes "$@" > $OUT/bench_${n}_$rep.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_${n}_$rep.log').read().strip().splitlines()[-1]); print('$n', $rep, d['ms_per_step'], d['roofline']['frac'])"
done; done

#!/bin/bash
# Whole-step A/B of the GEMM main-loop policy on one box, arms alternated: default (ring for the convs),
# ring for every GEMM (ACTH_GEMM_TILE_FLAGS=0x1000), ring also for dense products with K >= 1280 / 640
# (ACTH_GEMM_RING_K). Usage: tools/ab_step_ring.sh [rounds]
set -o pipefail
OUT=gpurun_out/r6_ab_ring
mkdir -p $OUT
ARGS="--steps 12 --warmup 2 --no-cpu-baseline --no-roofline --no-four-branch-compare --no-other-modes --no-fpb25 --no-fp16-compare"
for i in $(seq 1 ${1:-2}); do
  timeout -k 10 240 python3 -u bench.py $ARGS > $OUT/default_$i.log 2>&1 || exit $?
  ACTH_GEMM_TILE_FLAGS=0x1000 timeout -k 10 240 python3 -u bench.py $ARGS > $OUT/ringall_$i.log 2>&1 || exit $?
  ACTH_GEMM_RING_K=1280 timeout -k 10 240 python3 -u bench.py $ARGS > $OUT/ringk1280_$i.log 2>&1 || exit $?
  ACTH_GEMM_RING_K=640 timeout -k 10 240 python3 -u bench.py $ARGS > $OUT/ringk640_$i.log 2>&1 || exit $?
done
for f in $OUT/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done

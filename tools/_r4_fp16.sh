set -o pipefail
cd $GRAFT_REPO_ROOT
export ACTH_PARITY_LOG=gpurun_out/r4_fp16_parity.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_full_geometry_gpu.py -m gpu -k "fp16_budget" > gpurun_out/r4_fp16_test.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu > gpurun_out/r4_fp16_suite.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 5 --no-other-modes --no-four-branch-compare > gpurun_out/r4_bench_bf16.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 5 --no-other-modes --no-four-branch-compare --dtype fp16 > gpurun_out/r4_bench_fp16.log 2>&1
rc=$?
echo rc=$rc
tail -3 gpurun_out/r4_fp16_test.log gpurun_out/r4_fp16_suite.log
tail -1 gpurun_out/r4_bench_bf16.log gpurun_out/r4_bench_fp16.log
exit $rc

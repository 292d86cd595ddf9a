set -o pipefail
cd $GRAFT_REPO_ROOT
export ACTH_PARITY_LOG=gpurun_out/r4_parity.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_full_geometry_gpu.py -m gpu -k "${1:-c1_ or pipeline_call or loop25}" > gpurun_out/r4_pytest_parity.log 2>&1
echo rc=$?

set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4}
mkdir -p gpurun_out/$TAG
export ACTH_PARITY_LOG=gpurun_out/$TAG/parity.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
echo pytest rc=$rc
tail -3 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
echo smoke rc=$?

set -o pipefail
mkdir -p gpurun_out/mb19
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mb19/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mb19/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mb19/prof.log 2>&1

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or xattn" > gpurun_out/r4_pytest_gemm.log 2>&1
echo pytest rc=$?
tail -3 gpurun_out/r4_pytest_gemm.log
timeout -k 10 300 python tools/bench_gemm.py --tiles 0 --only 3,4,5,6,7,8,12,14,15 --residual --iters 20 > gpurun_out/r4_gemm_lds_res.log 2>&1 &&
timeout -k 10 300 python tools/gemm_stamps.py --only 3,6,12,5 --residual > gpurun_out/r4_gemm_lds_stamps.log 2>&1
echo rc=$?

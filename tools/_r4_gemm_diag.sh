set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_gemm.py --tiles 0 --only 3,4,5,6,7,8,12,14,15 --residual --iters 10 > gpurun_out/r4_gemm_res.log 2>&1 &&
timeout -k 10 300 python tools/bench_gemm.py --tiles 0 --only 3,4,5,6,7,8,12,14,15 --residual --iters 10 --flags 256 > gpurun_out/r4_gemm_res_noepi.log 2>&1 &&
timeout -k 10 300 python tools/gemm_stamps.py --only 3,6,12,5 --residual > gpurun_out/r4_gemm_stamps.log 2>&1
echo rc=$?

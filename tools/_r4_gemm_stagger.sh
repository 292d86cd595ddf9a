set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/bench_gemm.py --tiles 0 --only 3,4,5,6,7,8,12,14,15 --residual --iters 20 --stagger 0,1,2,3,4 > gpurun_out/r4_gemm_stagger_res.log 2>&1 &&
timeout -k 10 400 python tools/bench_gemm.py --tiles 0 --only 0,1,2,3,6,9,12,13 --iters 20 --stagger 0,1,2,3 > gpurun_out/r4_gemm_stagger_nores.log 2>&1
echo rc=$?

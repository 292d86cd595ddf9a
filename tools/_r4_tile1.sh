set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_gemm.py --tiles 0,1,2,3,4,5 --only 3,6,8,14,15 --iters 20 > gpurun_out/r4_tile1_nores.log 2>&1 &&
timeout -k 10 300 python tools/bench_gemm.py --tiles 0,1,2,3,4,5 --only 3,6,8,14,15 --iters 20 --residual > gpurun_out/r4_tile1_res.log 2>&1
rc=$?; cat gpurun_out/r4_tile1_nores.log gpurun_out/r4_tile1_res.log; exit $rc

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_gemm.py --tiles 0 --only 3,6,12,15 --iters 20 > gpurun_out/r4_gemm_nores.log 2>&1 &&
timeout -k 10 300 python tools/bench_gemm.py --tiles 0 --only 3,6,12,15 --iters 20 --sink > gpurun_out/r4_gemm_nores_sink.log 2>&1 &&
timeout -k 10 300 python tools/gemm_stamps.py --only 3,6,12 > gpurun_out/r4_gemm_stamps_nores.log 2>&1 &&
timeout -k 10 300 python tools/gemm_stamps.py --only 3,6,12 --sink > gpurun_out/r4_gemm_stamps_sink.log 2>&1
echo rc=$?

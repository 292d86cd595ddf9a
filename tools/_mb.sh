set -o pipefail
mkdir -p gpurun_out/mb22
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mb22/pytest.log 2>&1 || exit 1
for L in head pk pkstag; do
ACTH_LIB=$PWD/ab/lib_$L.so timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/mb22/attn_$L.log 2>&1 || exit 1
done
for L in head pk; do
ACTH_LIB=$PWD/ab/lib_$L.so timeout -k 10 300 python -u tools/bench_gemm.py --tiles 0 > gpurun_out/mb22/gemm_$L.log 2>&1 || exit 1
done

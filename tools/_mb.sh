set -o pipefail
mkdir -p gpurun_out/mb12
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in 0 256 512 1024; do
timeout -k 10 300 python -u tools/bench_gemm.py --tiles 5 --flags $f --only 2,4,6,12 > gpurun_out/mb12/f$f.log 2>&1 || exit 1
done

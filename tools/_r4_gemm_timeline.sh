set -o pipefail
cd $GRAFT_REPO_ROOT
for sg in 0 2 4; do
timeout -k 10 200 python tools/gemm_stamps.py --only 3,6 --residual --timeline --stagger $sg >> gpurun_out/r4_gemm_timeline2.log 2>&1 || exit 1
done
echo rc=$?

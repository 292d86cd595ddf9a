set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh r2fin && bash tools/profile_head.sh gpurun_out/r2fin_prof && \
timeout -k 10 200 python -u bench.py --mode 1 --no-cpu-baseline > gpurun_out/r2fin/bench_mode1.log 2>&1 && \
timeout -k 10 250 python -u bench.py --mode 2 --no-cpu-baseline > gpurun_out/r2fin/bench_mode2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --width 576 --no-cpu-baseline > gpurun_out/r2fin/bench_C1geom.log 2>&1
rc=$?
for f in bench bench_mode1 bench_mode2 bench_C1geom; do grep -o '"ms_per_step[^,]*' gpurun_out/r2fin/$f.log; done
exit $rc

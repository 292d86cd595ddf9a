#!/bin/bash
# Round-3 evidence at HEAD: GPU tests + smoke + bench line + kernel stats (gpu_check.sh), a kernel trace with
# the two HBM-traffic PMC passes (profile_head.sh), and the C1-geometry (576x576) bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3fin}
bash tools/gpu_check.sh $TAG && bash tools/profile_head.sh gpurun_out/${TAG}_prof && \
timeout -k 10 200 python -u bench.py --width 576 --no-cpu-baseline --no-other-modes > gpurun_out/$TAG/bench_C1geom.log 2>&1
rc=$?
for f in bench bench_C1geom; do grep -o '"ms_per_step[^,]*' gpurun_out/$TAG/$f.log; done
exit $rc

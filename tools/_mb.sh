set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_pass.sh gpurun_out/pmc2 && bash tools/gpu_check.sh s3d

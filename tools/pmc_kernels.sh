#!/bin/bash
# Counter evidence per kernel family: four rocprofv3 --pmc passes (each within the
# gfx950 per-pass slots: <= 8 SQ, <= 4 TCC) over tools/pmc_probe.py runs of one kernel at one shape.
# Usage: tools/pmc_kernels.sh <outdir> "<probe args>" ["<probe args>" ...]
#   e.g. tools/pmc_kernels.sh gpurun_out/pmc "gemm 3" "flash 56 9216 5" "scan 56 9249 640 20"
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
i=0
for PROBE in "$@"; do
  TAG=$(echo "$PROBE" | tr ' ' '_')
  mkdir -p "$OUT/$TAG"
  for p in 0 1 2 3; do
    timeout -s KILL 120 rocprofv3 --pmc ${PASSES[$p]} -f csv -d "$OUT/$TAG/p$p" -o run -- \
        python3 -u tools/pmc_probe.py $PROBE --iters 3 > "$OUT/$TAG/p$p.log" 2>&1 || { echo "pass $p of $PROBE failed"; exit 1; }
  done
  echo "done $PROBE"
done

#!/bin/bash
# GEMM main-loop counter passes: rocprofv3 --pmc over tools/pmc_probe.py runs of acth_gemm at
# one bench_gemm SHAPES index per probe, plus a kernel trace of torch.matmul (hipBLASLt) on the same shapes so the
# library's kernel name (tile / wave / MFMA parameters) sits beside our counters.
# Usage: tools/pmc_gemm.sh <outdir> <shape index> [<shape index> ...]
set -o pipefail
OUT=${1:-gpurun_out/pmc_gemm}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
  "SQ_WAVES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
)
for S in "$@"; do
  mkdir -p "$OUT/gemm_$S"
  for p in 0 1 2; do
    timeout -s KILL 120 rocprofv3 --pmc ${PASSES[$p]} -f csv -d "$OUT/gemm_$S/p$p" -o run -- \
        python3 -u tools/pmc_probe.py gemm $S --iters 3 > "$OUT/gemm_$S/p$p.log" 2>&1 || { echo "pass $p of gemm $S failed"; exit 1; }
  done
  echo "done gemm $S"
done

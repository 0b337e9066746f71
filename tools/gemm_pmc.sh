#!/bin/bash
# PMC passes over single GEMM configurations of tools/gemm_bench (case cfg pairs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gpmc
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for cc in "0 8" "8 2" "0 2"; do
  set -- $cc
  timeout -s KILL 60 rocprofv3 --pmc $P1 -d gpurun_out/gpmc -o p1_$1_$2 --output-format csv -- tools/gemm_bench $1 $2 > gpurun_out/gpmc/l1_$1_$2.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $P2 -d gpurun_out/gpmc -o p2_$1_$2 --output-format csv -- tools/gemm_bench $1 $2 > gpurun_out/gpmc/l2_$1_$2.log 2>&1 || exit 1
done

#!/bin/bash
# microbenchmarks + rocprof kernel durations of the LSTM step variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 tools/gemm_bench > gpurun_out/gb.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ubprof -o ub --output-format csv -- tools/lstm_step_bench > gpurun_out/ub.log 2>&1

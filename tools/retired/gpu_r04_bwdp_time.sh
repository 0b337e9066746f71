#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lstm_persist_gpu.py -k "persistent_lstm2_backward" > gpurun_out/t_bwdp.log 2>&1 || exit 1
: > gpurun_out/bwdp_time.txt
for ab in ${ABL:-0 8 16 32 1}; do
  AVC_BWDP_ABLATE=$ab timeout -k 10 120 python -u tools/lstm2_bwd_persist_time.py >> gpurun_out/bwdp_time.txt 2>&1 || exit 1
done

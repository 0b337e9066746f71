#!/bin/bash
# Round 6: the XCD-local lstm1 backward: its GPU tests, then alternating
# fp32 / bf16 step A/Bs against the split-K launches (gpurun_out/ab_env.txt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lstm_persist_gpu.py -k "xcd" > gpurun_out/xcdbwd_tests.txt 2>&1 || { tail -30 gpurun_out/xcdbwd_tests.txt; exit 1; }
tail -3 gpurun_out/xcdbwd_tests.txt
bash tools/ab_env.sh "AVC_LSTM_XCD_BWD=0" "AVC_LSTM_XCD_BWD=1" "AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_RESERVE=0" "AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_LDS=82432,AVC_XCD_BWD_RESERVE=0" || exit 1
AB_ARGS="--precision bf16" bash tools/ab_env.sh "AVC_LSTM_XCD_BWD=0" "AVC_LSTM_XCD_BWD=1" "AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_RESERVE=0" "AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_LDS=82432,AVC_XCD_BWD_RESERVE=0" || exit 1
cat gpurun_out/ab_env.txt

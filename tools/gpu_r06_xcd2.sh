#!/bin/bash
# Round 6: the XCD-local lstm1 backward again, now that the X6 GEMMs shortened the side stream
# (the main stream's lstm1 backward is on the critical path: side_timeline_fp32_x6.txt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
rm -f gpurun_out/ab_env.txt
bash tools/ab_env.sh "AVC_LSTM_XCD_BWD=0" "AVC_LSTM_XCD_BWD=1" "AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_LDS=49152" "AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_LDS=82432,AVC_XCD_BWD_RESERVE=0" || exit 1
AB_ARGS="--precision bf16" bash tools/ab_env.sh "AVC_LSTM_XCD_BWD=0" "AVC_LSTM_XCD_BWD=1" "AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_LDS=49152" || exit 1
cat gpurun_out/ab_env.txt
AVC_LSTM_XCD_BWD=1 timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_x6_xcd.txt 2>&1 || exit 1
tail -12 gpurun_out/side_fp32_x6_xcd.txt

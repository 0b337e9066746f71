#!/bin/bash
# Round 6: where the lstm1 backward's CUs go (side-stream timelines with / without the
# XCD-local backward) and the split-K depth of the per-step backward in the current schedule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_x0.txt 2>&1 || exit 1
AVC_LSTM_XCD_BWD=1 AVC_XCD_BWD_LDS=82432 AVC_XCD_BWD_RESERVE=0 timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_x1.txt 2>&1 || exit 1
bash tools/ab_env.sh "AVC_LSTM1_SPLITS=8" "AVC_LSTM1_SPLITS=4" "AVC_LSTM1_SPLITS=2" || exit 1
AB_ARGS="--precision bf16" bash tools/ab_env.sh "AVC_LSTM1_SPLITS=4" "AVC_LSTM1_SPLITS=2" "AVC_LSTM1_SPLITS=1" || exit 1
cat gpurun_out/ab_env.txt

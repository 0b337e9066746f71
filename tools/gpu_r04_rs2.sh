#!/bin/bash
# Row-split lstm2 forward: wavefront form under the row split, then whole-step A/B (fp32, bf16)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; rm -f gpurun_out/ab_env.txt
AVC_LSTM2_RS=1 timeout -k 10 180 python -u tools/lstm2_persist_time.py --ab AVC_LSTM2_LAG2 > gpurun_out/rs_lag_time.txt 2>&1 &&
bash tools/ab_env.sh "AVC_LSTM2_RS=0" "AVC_LSTM2_RS=1" &&
AB_ARGS="--precision bf16" bash tools/ab_env.sh "AVC_LSTM2_RS=0" "AVC_LSTM2_RS=1"

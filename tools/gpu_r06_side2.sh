#!/bin/bash
# Round 6: the side-stream tail with the XCD-local lstm1 backward: a second
# side stream for alternate flushes, the join batch on the main stream; alternating A/Bs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
X="AVC_LSTM_XCD_BWD=1,AVC_XCD_BWD_LDS=82432,AVC_XCD_BWD_RESERVE=0"
bash tools/ab_env.sh "AVC_SIDE_STREAMS=1" "AVC_SIDE_STREAMS=2" "AVC_JOIN_MAIN=1,AVC_SIDE_STREAMS=2" "$X" "$X,AVC_SIDE_STREAMS=2" "$X,AVC_SIDE_STREAMS=2,AVC_JOIN_MAIN=1" || exit 1
AVC_SIDE_STREAMS=2 timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_s2.txt 2>&1 || exit 1
AVC_SIDE_STREAMS=2 AVC_LSTM_XCD_BWD=1 AVC_XCD_BWD_LDS=82432 AVC_XCD_BWD_RESERVE=0 timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_s2x.txt 2>&1 || exit 1
AB_ARGS="--precision bf16" bash tools/ab_env.sh "AVC_SIDE_STREAMS=1" "AVC_SIDE_STREAMS=2" "$X" "$X,AVC_SIDE_STREAMS=2" || exit 1
cat gpurun_out/ab_env.txt

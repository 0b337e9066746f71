#!/bin/bash
# Prefetch depth of the fused LSTM backward steps (AVC_LSTM_PF = 2 / 3 / 4): isolated step
# times (tools/lstm_bwd_time.py, fp32 and bf16) and the training step (tools/ab_env.sh, fp32
# and bf16).  Results in gpurun_out/ab_lstm_pf.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
out=gpurun_out/ab_lstm_pf.txt; : > $out
for pf in 2 3 4 2; do
  for p in fp32 bf16; do
    AVC_LSTM_PF=$pf timeout -k 10 120 python tools/lstm_bwd_time.py $p > gpurun_out/lbt_pf.txt 2>/dev/null || exit 1
    grep fused gpurun_out/lbt_pf.txt | sed "s/^/PF=$pf /" >> $out
  done
done
rm -f gpurun_out/ab_env.txt
timeout -k 10 600 bash tools/ab_env.sh "AVC_LSTM_PF=2" "AVC_LSTM_PF=3" "AVC_LSTM_PF=4" || exit 1
AB_ARGS="--precision bf16" timeout -k 10 600 bash tools/ab_env.sh "AVC_LSTM_PF=2" "AVC_LSTM_PF=3" "AVC_LSTM_PF=4" || exit 1
cat gpurun_out/ab_env.txt >> $out

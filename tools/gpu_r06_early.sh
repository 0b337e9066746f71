#!/bin/bash
# Round 6: release decoder lstm2's weight gradients right after its backward (AVC_EARLY_FLUSH)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash tools/ab_env.sh "AVC_EARLY_FLUSH=0" "AVC_EARLY_FLUSH=1" "AVC_EARLY_FLUSH=2" || exit 1
AVC_EARLY_FLUSH=1 timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_early.txt 2>&1 || exit 1
AB_ARGS="--precision bf16" bash tools/ab_env.sh "AVC_EARLY_FLUSH=0" "AVC_EARLY_FLUSH=1" "AVC_EARLY_FLUSH=2" || exit 1
cat gpurun_out/ab_env.txt

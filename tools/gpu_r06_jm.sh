#!/bin/bash
# Round 6: join batch on the main stream with the XCD-local lstm1 backward default (fp32, bf16)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
rm -f gpurun_out/ab_env.txt
bash tools/ab_env.sh "AVC_JOIN_MAIN=0" "AVC_JOIN_MAIN=1" || exit 1
AB_ARGS="--precision bf16" bash tools/ab_env.sh "AVC_JOIN_MAIN=0" "AVC_JOIN_MAIN=1" || exit 1
cat gpurun_out/ab_env.txt
timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_final.txt 2>&1 || exit 1
tail -12 gpurun_out/side_fp32_final.txt

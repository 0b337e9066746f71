#!/bin/bash
# Round 6: the LSTM backward recurrences on the X6 split — tests, per-step time, step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lstm_bwd_fused_gpu.py tests/test_gemm_x6_gpu.py > gpurun_out/x6l_tests.txt 2>&1 || { tail -40 gpurun_out/x6l_tests.txt; exit 1; }
tail -2 gpurun_out/x6l_tests.txt
timeout -k 10 200 python tools/lstm_bwd_time.py fp32 > gpurun_out/lbt_x6.txt 2>&1 || { cat gpurun_out/lbt_x6.txt; exit 1; }
AVC_FP32_X6=0 timeout -k 10 200 python tools/lstm_bwd_time.py fp32 >> gpurun_out/lbt_x6.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/lbt_x6.txt
rm -f gpurun_out/ab_env.txt
bash tools/ab_env.sh "AVC_FP32_X6=0" "AVC_FP32_X6=1" || exit 1
cat gpurun_out/ab_env.txt

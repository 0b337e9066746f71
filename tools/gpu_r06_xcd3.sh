#!/bin/bash
# Round 6: the XCD-local lstm1 backward with a half-size fp32 slab (two 256-k rounds per step):
# tests, then its dynamic LDS 39744 (a GEMM workgroup fits beside it) vs 82432 (one per CU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lstm_persist_gpu.py -k xcd > gpurun_out/xcd3_tests.txt 2>&1 || { tail -30 gpurun_out/xcd3_tests.txt; exit 1; }
tail -1 gpurun_out/xcd3_tests.txt
rm -f gpurun_out/ab_env.txt
bash tools/ab_env.sh "AVC_XCD_BWD_LDS=82432" "AVC_XCD_BWD_LDS=39744" "AVC_XCD_BWD_LDS=49152" || exit 1
cat gpurun_out/ab_env.txt
AVC_XCD_BWD_LDS=39744 timeout -k 10 200 python tools/side_timeline.py fp32 20 > gpurun_out/side_fp32_xcd3.txt 2>&1 || exit 1
tail -12 gpurun_out/side_fp32_xcd3.txt

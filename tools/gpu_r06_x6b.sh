#!/bin/bash
# Round 6: X6 GEMMs with two stages in flight on the 256-row tile and the chip-filling split plan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/x6_tests.txt 2>&1 || { tail -40 gpurun_out/x6_tests.txt; exit 1; }
tail -2 gpurun_out/x6_tests.txt
timeout -k 10 200 python tools/gemm_x6_time.py > gpurun_out/x6_time.txt 2>&1 || { cat gpurun_out/x6_time.txt; exit 1; }
cat gpurun_out/x6_time.txt
bash tools/ab_env.sh "AVC_FP32_X6=0" "AVC_FP32_X6=1" || exit 1
cat gpurun_out/ab_env.txt

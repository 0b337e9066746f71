#!/bin/bash
# Round 6: X6 single-LDS-buffer 32-k tile (AVC_X6_BIG=3) vs the two-buffer 16-k tile: tests,
# isolated timing, step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
AVC_X6_BIG=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/x6sb_tests.txt 2>&1 || { tail -30 gpurun_out/x6sb_tests.txt; exit 1; }
tail -1 gpurun_out/x6sb_tests.txt
rm -f gpurun_out/x6_sb.txt
for v in 0 3; do
  echo "== AVC_X6_BIG=$v" >> gpurun_out/x6_sb.txt
  AVC_X6_BIG=$v timeout -k 10 200 python tools/gemm_x6_time.py >> gpurun_out/x6_sb.txt 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/x6_sb.txt
rm -f gpurun_out/ab_env.txt
bash tools/ab_env.sh "AVC_X6_BIG=0" "AVC_X6_BIG=3" || exit 1
cat gpurun_out/ab_env.txt

#!/bin/bash
# Round 6: four-stage X6 loop (sched 6 = main, sched 0 = xs0): tests, isolated timing, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/x6_tests.txt 2>&1 || { tail -30 gpurun_out/x6_tests.txt; exit 1; }
tail -1 gpurun_out/x6_tests.txt
rm -f gpurun_out/x6_d.txt
for v in main xs0; do
  L=""; [ $v != main ] && L=tools/pbin/libautovc_$v.so
  echo "== $v" >> gpurun_out/x6_d.txt
  env ${L:+AUTOVC_HIP_LIB=$L} timeout -k 10 200 python tools/gemm_x6_time.py >> gpurun_out/x6_d.txt 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/x6_d.txt
rm -f gpurun_out/ab_env.txt
bash tools/ab_env.sh "AVC_FP32_X6=1" "AUTOVC_HIP_LIB=tools/pbin/libautovc_xs0.so" || exit 1
cat gpurun_out/ab_env.txt

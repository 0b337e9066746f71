#!/bin/bash
# Round 6: X6 MFMA / conversion interleave variants (AVC_X6_SCHED 0 / 2 / 4 / 6): isolated timing,
# then the step for the main library (4) against 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for v in main xs0 xs2 xs6; do
  L=""; [ $v != main ] && L=tools/pbin/libautovc_$v.so
  echo "== $v" >> gpurun_out/x6_sched.txt
  env ${L:+AUTOVC_HIP_LIB=$L} timeout -k 10 200 python tools/gemm_x6_time.py >> gpurun_out/x6_sched.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/x6_sched.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/x6_tests.txt 2>&1 || { tail -40 gpurun_out/x6_tests.txt; exit 1; }
tail -1 gpurun_out/x6_tests.txt
bash tools/ab_env.sh "AUTOVC_HIP_LIB=tools/pbin/libautovc_xs0.so" "AVC_FP32_X6=1" || exit 1
cat gpurun_out/ab_env.txt

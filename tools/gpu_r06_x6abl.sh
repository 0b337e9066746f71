#!/bin/bash
# Round 6: X6 GEMM timing ablations (timing-only builds: no split arithmetic / hi*hi only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
rm -f gpurun_out/x6_abl.txt
for v in main xnocvt xmf1; do
  L=""; [ $v != main ] && L=tools/pbin/libautovc_$v.so
  echo "== $v" >> gpurun_out/x6_abl.txt
  env ${L:+AUTOVC_HIP_LIB=$L} timeout -k 10 200 python tools/gemm_x6_time.py >> gpurun_out/x6_abl.txt 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/x6_abl.txt

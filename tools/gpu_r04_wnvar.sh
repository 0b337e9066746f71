#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; : > gpurun_out/wnvar.txt
for v in default noPT noPTnoFetch noPTnoFetchnoRes; do
  echo "== $v" >> gpurun_out/wnvar.txt
  if [ $v = default ]; then L=; else L=tools/pbin/libautovc_$v.so; fi
  AUTOVC_HIP_LIB=${L:-$PWD/autovc_amd/libautovc_hip.so} WN_TC=4 timeout -k 10 200 python -u tools/wn_grid_ab.py >> gpurun_out/wnvar.txt 2>&1 || exit 1
done

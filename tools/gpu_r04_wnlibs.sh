#!/bin/bash
# All-CU WaveNet generation: in-tree library vs variant builds (AUTOVC_HIP_LIB), grid mode
# A/B per batch (tools/wn_grid_ab.py), e.g. bash tools/gpu_r04_wnlibs.sh tools/pbin/libautovc_nosleep.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
out=gpurun_out/wnlibs.txt; : > $out
for i in 1 2; do
  echo "== in-tree" >> $out
  WN_B=${WN_B:-1,2} timeout -k 10 200 python -u tools/wn_grid_ab.py >> $out 2>&1 || exit 1
  for lib in "$@"; do
    echo "== $lib" >> $out
    AUTOVC_HIP_LIB=$PWD/$lib WN_B=${WN_B:-1,2} timeout -k 10 200 python -u tools/wn_grid_ab.py >> $out 2>&1 || exit 1
  done
done

#!/bin/bash
# Alternating A/B of WaveNet generation: the in-tree library vs variant builds of it
# (AUTOVC_HIP_LIB=<path>), e.g. bash tools/wn_ab_libs.sh tools/build/libautovc_wn_pr16.so
set -o pipefail
cd "$(dirname "$0")/.."
for i in 1 2 3; do
  echo "in-tree:"; timeout -k 10 120 python tools/wn_time.py || exit 1
  for lib in "$@"; do
    echo "$lib:"; AUTOVC_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/wn_time.py || exit 1
  done
done

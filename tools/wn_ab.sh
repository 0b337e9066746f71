#!/bin/bash
# Alternating A/B of WaveNet generation: the working tree vs tools/ab_head (a copy of another
# revision's autovc_amd package with its built library).  Run on the GPU box.
set -o pipefail
cd "$(dirname "$0")/.."
for i in 1 2 3; do
  echo "new:";  timeout -k 10 120 python tools/wn_time.py || exit 1
  echo "head:"; WN_PKG_ROOT=$PWD/tools/ab_head timeout -k 10 120 python tools/wn_time.py || exit 1
done

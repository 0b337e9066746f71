#!/bin/bash
# time the front-end kernel of several library builds (var/*.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for so in var/*.so; do
  echo "== $so" >> gpurun_out/fe_var.log
  AUTOVC_HIP_LIB=$PWD/$so timeout -k 10 120 python tools/fe_probe.py >> gpurun_out/fe_var.log 2>&1 || exit 1
done

#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
AVC_WN_DEBUG=1 timeout -k 10 300 python -u tools/wn_grid_debug.py > gpurun_out/wndbg.txt 2>&1

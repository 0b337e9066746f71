#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 120 tools/pbin/granule_probe 20000 > gpurun_out/gprobe.txt 2>&1

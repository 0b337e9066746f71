#!/bin/bash
# All-CU WaveNet generation: the grid-vs-launches parity test, then the A/B timing only
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_wavenet_gpu.py \
  -k "grid_generation_matches" > gpurun_out/wngrid_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/wn_grid_ab.py > gpurun_out/wngrid_ab.txt 2>&1

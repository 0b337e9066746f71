#!/bin/bash
# All-CU WaveNet generation: parity tests (grid vs launches and vs the oracle), then the A/B timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_wavenet_gpu.py \
  -k "grid" > gpurun_out/wngrid_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/wn_grid_ab.py > gpurun_out/wngrid_ab.txt 2>&1

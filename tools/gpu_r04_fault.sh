#!/bin/bash
# Round-4 step-graph fault check, safest first; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
AUDIT_SIDE=1 tools/gpu_r04.sh audit && \
timeout -k 10 600 $T tests/test_solver_gpu.py -k "b64_graph_trajectory or (replays_without_host_sync and True)" > gpurun_out/t_side_on.log 2>&1 && \
AUDIT_SIDE=0 tools/gpu_r04.sh audit && \
timeout -k 10 900 $T tests/test_solver_gpu.py -k "replays_without_host_sync or step_bit_identical" > gpurun_out/t_graph.log 2>&1

#!/bin/bash
# A/B of the stacked lstm2 backward (AVC_LSTM2_BWD=1, default) against the layer-by-layer
# backward (=0): GPU tests of the LSTM paths first, then alternating bench runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_generator_gpu.py tests/test_solver_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_lstm2.log 2>&1 || exit 1
for v in 0 1 0 1; do
  AVC_LSTM2_BWD=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-wavenet --no-cpu-baseline --no-e2e --no-roofline --no-bf16 > gpurun_out/ab_l2_$v.json 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_l2_$v.json'));print(d['ms_per_step'], d['final_loss'])")" >> gpurun_out/ab_l2.txt
done

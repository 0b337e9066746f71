#!/bin/bash
# A/B of the split-K factor of the stacked lstm2 backward recurrence (AVC_LSTM2_SPLITS,
# 2 or 4), alternating bench runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for cfg in "4 0" "2 0" "4 0" "2 0"; do
  set -- $cfg
  AVC_LSTM2_SPLITS=$1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-wavenet --no-cpu-baseline --no-e2e --no-roofline --no-bf16 > gpurun_out/ab_s.json 2>/dev/null || exit 1
  echo "l2splits=$1 $(python -c "import json;d=json.load(open('gpurun_out/ab_s.json'));print(d['ms_per_step'], d['final_loss'])")" >> gpurun_out/ab_splits.txt
done

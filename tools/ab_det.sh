#!/bin/bash
# Determinism check of bench.py under environment/argument variants (tools only):
#   bash tools/ab_det.sh "ENV=.. ARGS" ...   each variant twice; final loss and ms/step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "$@"; do
    envs=$(echo "$cfg" | tr ' ' '\n' | grep '=' | tr '\n' ' ')
    args=$(echo "$cfg" | tr ' ' '\n' | grep -v '=' | tr '\n' ' ')
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-wavenet --no-cpu-baseline --no-e2e --no-roofline --no-bf16 $args > gpurun_out/ab_d.json 2>gpurun_out/ab_d.err || { tail -5 gpurun_out/ab_d.err; exit 1; }
    echo "$cfg | $(python -c "import json;d=json.load(open('gpurun_out/ab_d.json'));print(d['ms_per_step'], d['final_loss'])")" >> gpurun_out/ab_det.txt
  done
done

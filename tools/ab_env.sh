#!/bin/bash
# Alternating fp32 bench runs under environment overrides given as arguments, e.g.
#   bash tools/ab_env.sh "AVC_BLSTM_SIDE=1" "AVC_BLSTM_SIDE=2"
# (commas join several variables into one configuration: "AVC_A=1,AVC_B=0")
# Each configuration runs twice, interleaved; results in gpurun_out/ab_env.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "$@"; do
    env ${cfg//,/ } timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-wavenet --no-cpu-baseline --no-e2e --no-roofline --no-bf16 ${AB_ARGS} > gpurun_out/ab_e.json 2>/dev/null || exit 1
    echo "${AB_ARGS:+[$AB_ARGS] }$cfg $(python -c "import json;d=json.load(open('gpurun_out/ab_e.json'));print(d['ms_per_step'], d['final_loss'])")" >> gpurun_out/ab_env.txt
  done
done

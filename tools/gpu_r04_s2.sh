#!/bin/bash
# round 4, session 2: whole GPU suite, bench, what-if step timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
PYTEST_X= KEEP_GOING=1 tools/gpu_r04.sh tests; rc=$?
echo "tests rc=$rc" >> gpurun_out/status.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-wavenet --no-cpu-baseline --no-e2e > gpurun_out/bench_s2.json 2> gpurun_out/bench_s2.err || exit 1
timeout -k 10 300 python -u tools/step_whatif.py fp32 > gpurun_out/whatif.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/step_whatif.py bf16 >> gpurun_out/whatif.txt 2>&1 || exit 1

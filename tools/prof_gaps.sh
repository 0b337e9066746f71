#!/bin/bash
# rocprof kernel trace of the fp32 step + timeline summary (tools/trace_gaps.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/tl
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wavenet --no-e2e --no-roofline ${BENCH_ARGS} > gpurun_out/tl.log 2>&1 || exit 1
f=$(ls gpurun_out/tl/*kernel_trace.csv | head -1)
python tools/trace_gaps.py "$f" > gpurun_out/gaps.txt 2>&1
rc=$?
rm -f gpurun_out/tl/*kernel_trace.csv
exit $rc

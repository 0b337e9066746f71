#!/bin/bash
# Round 6 final measurement refresh: lstm2 forward PMC (the bench roofline's traffic), per-precision
# step accounting traces, rocprofv3 --stats of the default bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_f -o run --output-format csv -- python tools/lstm_pmc.py persist > gpurun_out/pmc_f.log 2>&1 || { tail gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_w -o run --output-format csv -- python tools/lstm_pmc.py persist > gpurun_out/pmc_w.log 2>&1 || { tail gpurun_out/pmc_w.log; exit 1; }
python tools/pmc_summarize.py gpurun_out/pmc_f gpurun_out/pmc_w persist > gpurun_out/lstm2_persist_pmc.json || exit 1
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w
cat gpurun_out/lstm2_persist_pmc.json
bash tools/gpu_r06_prof.sh trace_fp32,trace_bf16 || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o run --output-format csv -- python bench.py > gpurun_out/benchprof.json 2> gpurun_out/benchprof.err || { tail gpurun_out/benchprof.err; exit 1; }
rm -f gpurun_out/benchprof/run_kernel_trace.csv
find gpurun_out/benchprof -name '*kernel_trace.csv' -delete
ls gpurun_out/benchprof

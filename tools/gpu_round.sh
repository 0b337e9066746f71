#!/bin/bash
# One GPU-box session: tests, bench, rocprof kernel stats.  Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
run_tests() {
  if [ -n "$PYTEST_K" ]; then timeout -k 10 ${T_TESTS:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$PYTEST_K" > gpurun_out/tests.log 2>&1
  else timeout -k 10 ${T_TESTS:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; fi; }
run_bench() { timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; }
run_prof()  { timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wavenet --no-e2e > gpurun_out/prof.log 2>&1; }
case "$STEP" in
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  tb) run_tests && run_bench ;;
  bp) run_bench && run_prof ;;
  all) run_tests && run_bench && run_prof ;;
esac
rc=$?
echo "EXIT $rc" >> gpurun_out/status.txt
exit $rc

#!/bin/bash
# Round-6 GPU session steps; each GPU step has its own time limit and the chain stops at
# the first failure.  Usage: tools/gpu_r05.sh step[,step...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for STEP in ${1//,/ }; do
  echo "== $STEP $(date +%T)" >> gpurun_out/status.txt
  case "$STEP" in
    tests) timeout -k 10 ${T_TESTS:-1500} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu ${PYTEST_X--x} -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/tests.log 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
    benchprof) timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o run --output-format csv -- python bench.py ${BENCH_ARGS} > gpurun_out/benchprof.json 2> gpurun_out/benchprof.err && \
               rm -f gpurun_out/benchprof/run_kernel_trace.csv ;;   # the full bench's trace exceeds what gpurun copies back
    qbench) timeout -k 10 300 python bench.py --no-cpu-baseline --no-wavenet --no-e2e --no-roofline ${BENCH_ARGS} > gpurun_out/qbench${TAG}.json 2> gpurun_out/qbench${TAG}.err ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${PROF_TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wavenet --no-e2e --no-roofline ${PROF_ARGS} > gpurun_out/prof${PROF_TAG}.log 2>&1 ;;
    timeline) timeout -k 10 300 python -u tools/side_timeline.py fp32 ${TL_REPS:-10} > gpurun_out/side_timeline_fp32${TAG}.txt 2> gpurun_out/side_timeline.err && \
              timeout -k 10 300 python -u tools/side_timeline.py bf16 ${TL_REPS:-10} > gpurun_out/side_timeline_bf16${TAG}.txt 2>> gpurun_out/side_timeline.err ;;
    gemmcmp) timeout -k 10 300 python -u tools/gemm_vs_blas.py > gpurun_out/gemm_vs_blas.txt 2> gpurun_out/gemm_vs_blas.err ;;
    whatif) timeout -k 10 600 python -u tools/step_whatif.py fp32 > gpurun_out/step_whatif${TAG}.txt 2> gpurun_out/step_whatif.err && \
            timeout -k 10 600 python -u tools/step_whatif.py bf16 >> gpurun_out/step_whatif${TAG}.txt 2>> gpurun_out/step_whatif.err ;;
    abenv) timeout -k 10 ${T_AB:-900} bash tools/ab_env.sh $AB_CFGS 2> gpurun_out/ab_env.err ;;
    lbt) timeout -k 10 300 python -u tools/lstm_bwd_time.py fp32 > gpurun_out/lstm_bwd_time${TAG}.txt 2> gpurun_out/lbt.err && \
         timeout -k 10 300 python -u tools/lstm_bwd_time.py bf16 >> gpurun_out/lstm_bwd_time${TAG}.txt 2>> gpurun_out/lbt.err ;;
    lbtprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lbtprof${TAG} -o run --output-format csv -- python tools/lstm_bwd_time.py ${LBT_PREC:-fp32} > gpurun_out/lbtprof${TAG}.log 2>&1 ;;
    gemmpmc) for W in ours blas; do
               timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/gpmc_$W -o run --output-format csv -- python tools/gemm_pmc.py $W ${GEMM_SHAPE:-4096 1024 8192} 10 > gpurun_out/gpmc_$W.log 2>&1 || exit 1
               timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/gpmc2_$W -o run --output-format csv -- python tools/gemm_pmc.py $W ${GEMM_SHAPE:-4096 1024 8192} 10 > gpurun_out/gpmc2_$W.log 2>&1 || exit 1
             done ;;
    bwdpmc) for P in fp32 bf16; do
               timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/bpmc_f_$P -o run --output-format csv -- python tools/lstm_bwd_time.py $P > gpurun_out/bpmc_f_$P.log 2>&1 || exit 1
               timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/bpmc_h_$P -o run --output-format csv -- python tools/lstm_bwd_time.py $P > gpurun_out/bpmc_h_$P.log 2>&1 || exit 1
             done ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
  rc=$?
  echo "   $STEP rc=$rc $(date +%T)" >> gpurun_out/status.txt
  case $rc in 0) ;; 1|2) [ -n "$KEEP_GOING" ] || exit $rc ;; *) exit $rc ;; esac
done
exit 0

#!/bin/bash
# Round-4 GPU session steps; each GPU step has its own time limit and the chain stops at
# the first failure.  Usage: tools/gpu_r04.sh step[,step...]
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
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${PROF_TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wavenet --no-e2e --no-roofline ${PROF_ARGS} > gpurun_out/prof${PROF_TAG}.log 2>&1 ;;
    wnprof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/wnprof -o run --output-format csv -- python tools/wn_pmc.py 4 > gpurun_out/wnprof.log 2>&1 ;;
    wnpmc) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/wnpmc_f -o run --output-format csv -- python tools/wn_pmc.py 1 > gpurun_out/wnpmc_f.log 2>&1 && \
           timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/wnpmc_w -o run --output-format csv -- python tools/wn_pmc.py 1 > gpurun_out/wnpmc_w.log 2>&1 && \
           python tools/wn_pmc_summarize.py gpurun_out/wnpmc_f gpurun_out/wnpmc_w 256 > gpurun_out/wavenet_pmc.json && \
           rm -f gpurun_out/wnpmc_f/*/*.csv.bak ;;
    lppmc) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/lppmc_f -o run --output-format csv -- python tools/lstm_pmc.py persist > gpurun_out/lppmc_f.log 2>&1 && \
           timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/lppmc_w -o run --output-format csv -- python tools/lstm_pmc.py persist > gpurun_out/lppmc_w.log 2>&1 && \
           python tools/pmc_summarize.py gpurun_out/lppmc_f gpurun_out/lppmc_w persist > gpurun_out/lstm2_persist_pmc.json ;;
    wnsweep) timeout -k 10 600 python tools/wavenet_bench.py 16 8 > gpurun_out/wnsweep.log 2>&1 ;;
    det) timeout -k 10 ${T_DET:-600} python -u tools/det_probe.py ${DET_B:-64} ${DET_STEPS:-6} ${DET_VARIANTS:-graph=1,stream=0 graph=1,stream=1} > gpurun_out/det.log 2> gpurun_out/det.err ;;
    bench2) timeout -k 10 900 python bench.py --gpus 2 ${BENCH_ARGS} > gpurun_out/bench2.json 2> gpurun_out/bench2.err ;;
    blpmc) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/blpmc_f -o run --output-format csv -- python tools/lstm_pmc.py blstm > gpurun_out/blpmc_f.log 2>&1 && \
           timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/blpmc_w -o run --output-format csv -- python tools/lstm_pmc.py blstm > gpurun_out/blpmc_w.log 2>&1 && \
           python tools/pmc_summarize.py gpurun_out/blpmc_f gpurun_out/blpmc_w blstm_fwd > gpurun_out/blstm_fwd_pmc.json && \
           python tools/pmc_summarize.py gpurun_out/blpmc_f gpurun_out/blpmc_w blstm_bwd > gpurun_out/blstm_bwd_pmc.json && \
           timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/xpmc_f -o run --output-format csv -- python tools/lstm_pmc.py xcd > gpurun_out/xpmc_f.log 2>&1 && \
           timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/xpmc_w -o run --output-format csv -- python tools/lstm_pmc.py xcd > gpurun_out/xpmc_w.log 2>&1 && \
           python tools/pmc_summarize.py gpurun_out/xpmc_f gpurun_out/xpmc_w xcd > gpurun_out/lstm_xcd_pmc.json ;;
    wnpersist) timeout -k 10 120 tools/pbin/wn_persist_ubench > gpurun_out/wn_persist_ubench.txt 2>&1 && \
               timeout -k 10 300 tools/pbin/chain_ubench > gpurun_out/chain_ubench.txt 2>&1 ;;
    audit) timeout -k 10 300 python -u tools/graph_ptr_audit.py ${AUDIT_B:-64} ${AUDIT_SIDE:-1} ${AUDIT_PREC:-fp32} >> gpurun_out/audit.log 2>&1 ;;
    bench_nss) AVC_GRAD_STREAM=0 timeout -k 10 300 python bench.py --steps 25 --warmup 5 --no-wavenet --no-cpu-baseline --no-e2e --no-roofline > gpurun_out/bench_grad_stream0.json 2> gpurun_out/bench_grad_stream0.err ;;
    ring) timeout -k 10 120 python -u tools/graph_ring_probe.py ${RING_N:-2000} ${RING_R:-1,2,4,8,16,32} ${RING_F:-1,0} > gpurun_out/ring.log 2>&1 ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
  rc=$?
  echo "   $STEP rc=$rc $(date +%T)" >> gpurun_out/status.txt
  case $rc in 0) ;; 1|2) [ -n "$KEEP_GOING" ] || exit $rc ;; *) exit $rc ;; esac
done
exit 0

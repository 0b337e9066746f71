#!/bin/bash
# Round-6 measurement refresh (VERDICT r5 item 3 and item 2's counters): per-precision kernel
# traces of the bench command, PMC passes of the fused lstm2 backward step (fp32, bf16) and of the
# WaveNet generation.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wavenet --no-e2e --no-roofline --no-bf16"
run() { echo "== $1 $(date +%T)" >> gpurun_out/prof_status.txt; }
for STEP in ${1//,/ }; do
  run "$STEP"
  case "$STEP" in
    trace_fp32|trace_bf16)
        P=${STEP#trace_}; EXTRA=""; [ $P = bf16 ] && EXTRA="--precision bf16"
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$P -o run --output-format csv -- $BENCH $EXTRA > gpurun_out/tr_$P.log 2>&1 && \
        python tools/step_accounting.py "$(find gpurun_out/tr_$P -name '*kernel_trace.csv' | head -1)" > gpurun_out/step_accounting_${P}_r06.txt && \
        find gpurun_out/tr_$P -name '*kernel_trace.csv' -delete ;;
    bwdpmc) for P in fp32 bf16; do
          timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/bp_f_$P -o run --output-format csv -- python tools/lstm_bwd_time.py $P > gpurun_out/bp_f_$P.log 2>&1 || exit 1
          timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/bp_w_$P -o run --output-format csv -- python tools/lstm_bwd_time.py $P > gpurun_out/bp_w_$P.log 2>&1 || exit 1
          timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/bp_s_$P -o run --output-format csv -- python tools/lstm_bwd_time.py $P > gpurun_out/bp_s_$P.log 2>&1 || exit 1
          timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/bp_g_$P -o run --output-format csv -- python tools/lstm_bwd_time.py $P > gpurun_out/bp_g_$P.log 2>&1 || exit 1
          python tools/pmc_kernel_summary.py lstm2_bwd_fused_kernel gpurun_out/bp_f_$P gpurun_out/bp_w_$P gpurun_out/bp_s_$P gpurun_out/bp_g_$P --label "lstm2 fused backward step, $P, tools/lstm_bwd_time.py" > gpurun_out/lstm2_bwd_fused_pmc_$P.json || exit 1
          python tools/pmc_kernel_summary.py lstm_bwd_fused_kernel gpurun_out/bp_f_$P gpurun_out/bp_w_$P gpurun_out/bp_s_$P gpurun_out/bp_g_$P --label "lstm1 fused backward step, $P" > gpurun_out/lstm_bwd_fused_pmc_$P.json || exit 1
          rm -rf gpurun_out/bp_?_$P
        done ;;
    wnpmc) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/wp_f -o run --output-format csv -- python tools/wn_pmc.py 4 8 > gpurun_out/wp_f.log 2>&1 && \
           timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/wp_w -o run --output-format csv -- python tools/wn_pmc.py 4 8 > gpurun_out/wp_w.log 2>&1 && \
           timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/wp1_f -o run --output-format csv -- python tools/wn_pmc.py 4 1 > gpurun_out/wp1_f.log 2>&1 && \
           timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/wp1_w -o run --output-format csv -- python tools/wn_pmc.py 4 1 > gpurun_out/wp1_w.log 2>&1 && \
           python tools/pmc_kernel_summary.py wn_pipe_kernel gpurun_out/wp_f gpurun_out/wp_w --label "wn_pipe_kernel, 8 utterances x 1024 sample steps (one launch per 128-step chunk)" > gpurun_out/wavenet_pipe_pmc_b8.json && \
           python tools/pmc_kernel_summary.py wn_pipe_kernel gpurun_out/wp1_f gpurun_out/wp1_w --label "wn_pipe_kernel, 1 utterance x 1024 sample steps" > gpurun_out/wavenet_pipe_pmc_b1.json && \
           rm -rf gpurun_out/wp_f gpurun_out/wp_w gpurun_out/wp1_f gpurun_out/wp1_w ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
  rc=$?
  echo "   $STEP rc=$rc $(date +%T)" >> gpurun_out/prof_status.txt
  [ $rc -eq 0 ] || exit $rc
done

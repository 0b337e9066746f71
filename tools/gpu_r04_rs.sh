#!/bin/bash
# Row-split lstm2 forward: parity tests, then the A/B timing (AVC_LSTM2_RS=0/1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lstm_persist_gpu.py \
  -k "row_split or persistent_matches or bf16_persistent" > gpurun_out/rs_tests.txt 2>&1 &&
timeout -k 10 180 python -u tools/lstm2_persist_time.py --ab AVC_LSTM2_RS > gpurun_out/rs_time.txt 2>&1

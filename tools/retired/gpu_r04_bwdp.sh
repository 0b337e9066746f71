set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_lstm_persist_gpu.py -k "persistent_lstm2_backward" > gpurun_out/t_bwdp.log 2>&1 && \
timeout -k 10 600 $T tests/test_solver_gpu.py tests/test_generator_gpu.py -k "b64 or full_size or replays_without or step_bit_identical" > gpurun_out/t_bwdp_solver.log 2>&1 && \
timeout -k 10 300 python bench.py --no-wavenet --no-cpu-baseline --no-e2e > gpurun_out/bench_bwdp.json 2> gpurun_out/bench_bwdp.err && \
AVC_LSTM2_BWD_PERSIST=0 timeout -k 10 300 python bench.py --no-wavenet --no-cpu-baseline --no-e2e --no-roofline > gpurun_out/bench_bwdp0.json 2>> gpurun_out/bench_bwdp.err && \
AVC_LSTM2_BWD_FLUSH=beside timeout -k 10 300 python bench.py --no-wavenet --no-cpu-baseline --no-e2e --no-roofline > gpurun_out/bench_bwdp_beside.json 2>> gpurun_out/bench_bwdp.err

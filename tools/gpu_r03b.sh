#!/bin/bash
# Round-3 session-2 GPU call: GPU tests (a failing test does not stop the call; a crash,
# abort or time limit does), then A/B runs and the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
PYTEST_X= tools/gpu_r03.sh tests; rc=$?
echo "tests rc=$rc" >> gpurun_out/status.txt
[ $rc -le 1 ] || exit $rc
for ab in "$@"; do
  case "$ab" in
    bench) tools/gpu_r03.sh bench || exit $? ;;
    *) eval "$ab" || exit $? ;;
  esac
done
exit 0

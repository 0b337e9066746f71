#!/bin/bash
# Tile configurations of the fused LSTM backward steps (k chunk / waves / chunks in flight),
# timed in isolation with tools/lstm_bwd_time.py (fp32, bf16).  build on the CPU, run on the GPU.
set -e
cd "$(dirname "$0")/.."
CFGS="nw4:-DAVC_BNW=4 d3:-DAVC_BD=3 nw4d3:-DAVC_BNW=4,-DAVC_BD=3 k128nw4:-DAVC_BKCH=128,-DAVC_BNW=4 k32:-DAVC_BKCH=32"
if [ "$1" = build ]; then
  for c in $CFGS; do f=${c#*:}; bash tools/build_variant.sh bt_${c%%:*} ${f//,/ } > /dev/null; done
  exit 0
fi
for P in fp32 bf16; do
  echo "== product ($P)"; timeout -k 10 120 python tools/lstm_bwd_time.py $P | grep fused
  for c in $CFGS; do
    echo "== ${c%%:*} ($P)"; AUTOVC_HIP_LIB=tools/pbin/libautovc_bt_${c%%:*}.so timeout -k 10 120 python tools/lstm_bwd_time.py $P | grep fused
  done
done

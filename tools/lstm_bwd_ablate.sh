#!/bin/bash
# Timing ablations of the fused lstm2 backward step (where its 22.8 / 13.0 us
# go).  Builds timing-only variants (wrong results by design) and times each with
# tools/lstm_bwd_time.py, fp32 and bf16.  Build on the CPU: bash tools/lstm_bwd_ablate.sh build;
# run on the GPU: bash tools/lstm_bwd_ablate.sh run > gpurun_out/lstm2_bwd_ablate.txt
set -e
cd "$(dirname "$0")/.."
VARIANTS="empty:-DAVC_ABL_EMPTY nomfma:-DAVC_ABL_NOMFMA noarrive:-DAVC_ABL_NOARRIVE notail:-DAVC_ABL_NOTAIL"
if [ "$1" = build ]; then
  for v in $VARIANTS; do bash tools/build_variant.sh abl_${v%%:*} ${v#*:} > /dev/null; done
  exit 0
fi
for P in fp32 bf16; do
  echo "== product library ($P)"; timeout -k 10 120 python tools/lstm_bwd_time.py $P | grep lstm2
  for v in $VARIANTS; do
    echo "== ${v%%:*} ($P)"; AUTOVC_HIP_LIB=tools/pbin/libautovc_abl_${v%%:*}.so timeout -k 10 120 python tools/lstm_bwd_time.py $P | grep "lstm2 fused"
  done
done

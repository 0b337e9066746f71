#!/bin/bash
# Ablations / variants of the persistent lstm2 forward (lstm2_persist.hip):
#   bash tools/lp_ablate.sh build      (build container)      bash tools/lp_ablate.sh run   (GPU box)
# LP_MODES: LP_ABLATE modes (1 no barrier, 2 no products, 3 no h loads, 4 no epilogue);
# LP_VARIANTS: space-separated name=defines variants (defines comma-separated), e.g.
#   LP_VARIANTS="w2=-DLP_PWIN=2 vg=-DLP_W1_LDS=0,-DLP_PWIN=2"
set -o pipefail
cd "$(dirname "$0")/.."
MODES="${LP_MODES:-1 2 3 4}"
VARIANTS="${LP_VARIANTS:-}"
libs=()
for m in $MODES; do libs+=("ab$m=-DLP_ABLATE=$m"); done
for v in $VARIANTS; do libs+=("$v"); done
if [ "$1" = build ]; then
  mkdir -p tools/build
  objs=$(ls autovc_amd/csrc/build/*.o | grep -v '/lstm2_persist.o$')
  for e in "${libs[@]}"; do
    name=${e%%=*}; defs=${e#*=}; defs=${defs//,/ }
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
      -Iinclude $defs -x hip -c autovc_amd/csrc/lstm2_persist.hip -o tools/build/lp_$name.o || exit 1
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/build/libautovc_lp_$name.so $objs tools/build/lp_$name.o || exit 1
  done
  echo "${libs[@]}" > tools/build/lp_libs.txt
  exit 0
fi
echo "product"; timeout -k 10 120 python tools/lstm2_persist_time.py || exit 1
for e in $(cat tools/build/lp_libs.txt); do
  name=${e%%=*}
  echo "$e"; AUTOVC_HIP_LIB=$PWD/tools/build/libautovc_lp_$name.so timeout -k 10 120 python tools/lstm2_persist_time.py || exit 1
done

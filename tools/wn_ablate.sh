#!/bin/bash
# Diagnostic ablation libraries of the WaveNet step kernels (WN_ABLATE in wavenet.hip):
#   build (in the build container):  bash tools/wn_ablate.sh build
#   run   (on the GPU box):           bash tools/wn_ablate.sh run  > gpurun_out/wn_ablate.txt
set -o pipefail
cd "$(dirname "$0")/.."
MODES="${WN_MODES:-1 2 3 4 5 6 7 8 9 10}"
if [ "$1" = build ]; then
  mkdir -p tools/build
  objs=$(ls autovc_amd/csrc/build/*.o | grep -v '/wavenet.o$')
  for m in $MODES; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
      -Iinclude -DWN_ABLATE=$m -x hip -c autovc_amd/csrc/wavenet.hip -o tools/build/wavenet_ab$m.o || exit 1
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/build/libautovc_wn_ab$m.so $objs tools/build/wavenet_ab$m.o || exit 1
  done
  exit 0
fi
echo "mode 0 (product)"; timeout -k 10 120 python tools/wn_time.py || exit 1
for m in $MODES; do
  echo "mode $m"; AUTOVC_HIP_LIB=$PWD/tools/build/libautovc_wn_ab$m.so timeout -k 10 120 python tools/wn_time.py || exit 1
done

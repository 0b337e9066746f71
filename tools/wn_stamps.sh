#!/bin/bash
# Diagnostic timeline library of the WaveNet step kernels (WN_STAMP in wavenet.hip):
#   build (in the build container):  bash tools/wn_stamps.sh build
#   run   (on the GPU box):           bash tools/wn_stamps.sh run > gpurun_out/wn_stamps.txt
set -o pipefail
cd "$(dirname "$0")/.."
if [ "$1" = build ]; then
  mkdir -p tools/build
  objs=$(ls autovc_amd/csrc/build/*.o | grep -v '/wavenet.o$')
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
    -Iinclude -DWN_STAMP=1 -x hip -c autovc_amd/csrc/wavenet.hip -o tools/build/wavenet_stamp.o || exit 1
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/build/libautovc_wn_stamp.so $objs tools/build/wavenet_stamp.o
  exit $?
fi
AUTOVC_HIP_LIB=$PWD/tools/build/libautovc_wn_stamp.so timeout -k 10 180 python tools/wn_stamps.py

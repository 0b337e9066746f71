#!/bin/bash
# The phase-trace variant of the library (tools only): wavenet.hip with AVC_WN_GRID_TRACE, the
# rest from the regular build; output tools/pbin/libautovc_hip_trace.so (load it with
# AUTOVC_HIP_LIB=...).
set -euo pipefail
cd "$(dirname "$0")/../autovc_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../tools/pbin
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
  -I../../include -DAVC_WN_GRID_TRACE -x hip -c wavenet.hip -o ../../tools/pbin/wavenet_trace.o
objs=$(ls build/*.o | grep -v '^build/wavenet.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/pbin/libautovc_hip_trace.so $objs \
  ../../tools/pbin/wavenet_trace.o

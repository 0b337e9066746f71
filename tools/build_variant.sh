#!/bin/bash
# Build a variant of libautovc_hip.so with extra -D flags for A/B runs (tools only):
#   tools/build_variant.sh NAME "-DWINO_TPW=4 -DWINO_WAVES=4"  ->  tools/pbin/libautovc_NAME.so
# then AUTOVC_HIP_LIB=tools/pbin/libautovc_NAME.so selects it (autovc_amd/_lib.py).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
rm -rf tools/pbin/obj_$name; mkdir -p tools/pbin/obj_$name
pids=()
for f in autovc_amd/csrc/capi.cpp autovc_amd/csrc/*.hip; do
  b=$(basename "${f%.*}")
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
    -Iinclude $* -x hip -c "$f" -o tools/pbin/obj_$name/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "build of variant $name failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/pbin/libautovc_$name.so tools/pbin/obj_$name/*.o
rm -rf tools/pbin/obj_$name
echo tools/pbin/libautovc_$name.so

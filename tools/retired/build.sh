#!/bin/bash
# Compile the retired variants' sources (as of commit 226dc43, round 4) for gfx950 on the CPU:
# object files only, never linked into the product library.   bash tools/retired/build.sh
set -e
cd "$(dirname "$0")/../.."
REV=${RETIRED_REV:-226dc43}
OUT=tools/retired/build
rm -rf "$OUT" && mkdir -p "$OUT/src/autovc_amd/csrc" "$OUT/src/include"
for f in common.h bn_finalize.h twiddle1024.h lstm2_persist.hip wavenet.hip winograd.hip gemm.hip; do
  git show "$REV:autovc_amd/csrc/$f" > "$OUT/src/autovc_amd/csrc/$f"
done
git show "$REV:include/autovc_hip.h" > "$OUT/src/include/autovc_hip.h"
for f in lstm2_persist wavenet winograd gemm; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I"$OUT/src/include" \
    -x hip -c "$OUT/src/autovc_amd/csrc/$f.hip" -o "$OUT/$f.o" &
done
wait
# the trace build of the all-CU WaveNet kernel
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -DAVC_WN_GRID_TRACE \
  -I"$OUT/src/include" -x hip -c "$OUT/src/autovc_amd/csrc/wavenet.hip" -o "$OUT/wavenet_trace.o"
# the mirrored all-gather (round 5, commit d196949)
MREV=${MIRROR_REV:-d196949}
mkdir -p "$OUT/mirror/autovc_amd/csrc" "$OUT/mirror/include"
for f in common.h twiddle1024.h wavenet.hip; do
  git show "$MREV:autovc_amd/csrc/$f" > "$OUT/mirror/autovc_amd/csrc/$f"
done
git show "$MREV:include/autovc_hip.h" > "$OUT/mirror/include/autovc_hip.h"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I"$OUT/mirror/include" \
  -x hip -c "$OUT/mirror/autovc_amd/csrc/wavenet.hip" -o "$OUT/wavenet_mirror.o"
# the LDS-DMA weight-gradient GEMM (round 5, commit 9d01bc2)
CREV=${CC_REV:-9d01bc2}
mkdir -p "$OUT/cc/autovc_amd/csrc" "$OUT/cc/include"
for f in common.h gemm.hip; do
  git show "$CREV:autovc_amd/csrc/$f" > "$OUT/cc/autovc_amd/csrc/$f"
done
git show "$CREV:include/autovc_hip.h" > "$OUT/cc/include/autovc_hip.h"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I"$OUT/cc/include" \
  -x hip -c "$OUT/cc/autovc_amd/csrc/gemm.hip" -o "$OUT/gemm_cc.o"
ls -la "$OUT"/*.o

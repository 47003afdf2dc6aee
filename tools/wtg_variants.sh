#!/bin/bash
# Builds libncgpu.so variants of the window tempogram kernel (window_stage.hip knobs
# NC_WT_SEG / NC_WT_PAIR / NC_WT_SKIP) into tools/var/<name>/ for tools/wtg_bench.py.
set -e
cd "$(dirname "$0")/.."
PKG=nightcore-to-flac-analyzer_amd
make -s -C $PKG -j8 ARCH=gfx950
for spec in "seg1_pair1:-DNC_WT_SEG=1 -DNC_WT_PAIR=1" "seg1_pair2:-DNC_WT_SEG=1 -DNC_WT_PAIR=2" \
            "seg2_pair2:-DNC_WT_SEG=2 -DNC_WT_PAIR=2" "seg4_pair2:-DNC_WT_SEG=4 -DNC_WT_PAIR=2" \
            "seg2_pair1:-DNC_WT_SEG=2 -DNC_WT_PAIR=1" \
            "skip1:-DNC_WT_SEG=1 -DNC_WT_PAIR=1 -DNC_WT_SKIP=1" "skip2:-DNC_WT_SEG=1 -DNC_WT_PAIR=1 -DNC_WT_SKIP=2"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p tools/var/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -x hip -c $PKG/csrc/window_stage.hip \
    -o tools/var/$name/window_stage.o
  objs=$(ls $PKG/build/*.o | grep -v window_stage.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/var/$name/libncgpu.so $objs tools/var/$name/window_stage.o
done
echo built

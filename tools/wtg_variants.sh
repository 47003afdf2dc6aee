#!/bin/bash
# Builds libncgpu.so variants of the window tempogram kernel (window_stage.hip knobs
# NC_WT_THREADS / NC_WT_STAGE, nc_tgcorr.h NC_TGC_LB) into tools/var/<name>/ for
# tools/wtg_bench.py.   usage: tools/wtg_variants.sh "name:-DFLAG=.. -DFLAG=.." ...
set -e
cd "$(dirname "$0")/.."
PKG=nightcore-to-flac-analyzer_amd
make -s -C $PKG -j8 ARCH=gfx950
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p tools/var/$name
  /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950 $flags -x hip \
    -c $PKG/csrc/window_stage.hip -o tools/var/$name/window_stage.o
  objs=$(ls $PKG/build/*.o | grep -v window_stage.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/var/$name/libncgpu.so $objs tools/var/$name/window_stage.o
done
echo built

#!/bin/bash
# Builds libncgpu.so variants: tools/var_build.sh "name:a.hip,b.hip:-DFLAGS" ... -> tools/var/<name>/libncgpu.so
# (the listed sources are rebuilt with the extra flags, every other object is the in-tree build)
set -e
cd "$(dirname "$0")/.."
PKG=nightcore-to-flac-analyzer_amd
make -s -C $PKG -j8 ARCH=gfx950
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; files=${rest%%:*}; flags=${rest#*:}
  mkdir -p tools/var/$name
  objs=$(ls $PKG/build/*.o)
  for file in ${files//,/ }; do
    base=$(basename $file .hip)
    /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950 $flags -x hip -c $PKG/csrc/$file -o tools/var/$name/$base.o
    objs=$(echo "$objs" | grep -v "/$base.o")
    objs="$objs tools/var/$name/$base.o"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/var/$name/libncgpu.so $objs
done
echo built

#!/bin/bash
# Builds libncgpu.so from the in-tree objects with some sources taken from a git revision:
#   tools/var_build_rev.sh NAME REV file.hip [file.hip ...]  -> tools/var/NAME/libncgpu.so
# (headers come from the working tree: only for revisions whose headers are unchanged)
set -e
cd "$(dirname "$0")/.."
PKG=nightcore-to-flac-analyzer_amd
name=$1; rev=$2; shift 2
make -s -C $PKG -j8 ARCH=gfx950
mkdir -p tools/var/$name
objs=$(ls $PKG/build/*.o)
for file in "$@"; do
  base=$(basename $file .hip)
  git show $rev:$PKG/csrc/$file > tools/var/$name/$file
  /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950 -I $PKG/csrc -I include \
    -x hip -c tools/var/$name/$file -o tools/var/$name/$base.o
  objs=$(echo "$objs" | grep -v "/$base.o")
  objs="$objs tools/var/$name/$base.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/var/$name/libncgpu.so $objs
echo built $name

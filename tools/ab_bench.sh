#!/bin/bash
# A/B step timing of library builds in one GPU session: alternates bench.py runs (timed
# region only) over the in-tree library and each NCGPU_LIB given.
#   usage: tools/ab_bench.sh OUTDIR ROUNDS lib1.so [lib2.so ...]
set -o pipefail
O=$1; N=$2; shift 2
mkdir -p $O
for i in $(seq $N); do
  for lib in intree "$@"; do
    tag=$(basename $(dirname $lib))
    [ $lib = intree ] && tag=intree
    if [ $lib = intree ]; then
      timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload --no-ibi > $O/$tag.$i.json 2> $O/$tag.$i.err || { echo "bench $tag failed"; tail -5 $O/$tag.$i.err; exit 1; }
    else
      NCGPU_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload --no-ibi > $O/$tag.$i.json 2> $O/$tag.$i.err || { echo "bench $tag failed"; tail -5 $O/$tag.$i.err; exit 1; }
    fi
    python3 -c "import json; d=json.load(open('$O/$tag.$i.json')); print('$tag', $i, round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
  done
done

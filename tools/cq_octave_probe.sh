set -o pipefail
O=gpurun_out/r6cq
mkdir -p $O
B=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
timeout -k 10 500 python3 -u tools/var_bench.py $B tools/var/o0/libncgpu.so tools/var/o0nobw/libncgpu.so tools/var/o1/libncgpu.so tools/var/o1nobw/libncgpu.so tools/var/allnobw0/libncgpu.so > $O/var_bench.txt 2>&1 || { echo "var bench failed"; tail -20 $O/var_bench.txt; exit 1; }
cat $O/var_bench.txt

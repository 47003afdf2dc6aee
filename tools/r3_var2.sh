set -o pipefail
O=gpurun_out/r3_var2
mkdir -p $O
timeout -k 10 300 python3 tools/var_bench.py tools/var/base/libncgpu.so tools/var/incloc/libncgpu.so tools/var/tpdefer/libncgpu.so tools/var/prolog/libncgpu.so > $O/var.log 2>&1 || { echo "var failed"; tail -20 $O/var.log; exit 1; }
grep -v amdgpu.ids $O/var.log

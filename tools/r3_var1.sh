set -o pipefail
O=gpurun_out/r3_var1
mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python3 tools/var_bench.py tools/var/base/libncgpu.so tools/var/melu/libncgpu.so tools/var/cl_nowait/libncgpu.so >> $O/var.log 2>&1 || { echo "var failed"; tail -20 $O/var.log; exit 1; }
done
cat $O/var.log | grep -v amdgpu.ids

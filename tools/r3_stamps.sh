set -o pipefail
O=gpurun_out/r3_stamps
mkdir -p $O
timeout -k 10 300 python3 tools/var_bench.py tools/var/cur/libncgpu.so tools/var/tpstamps/libncgpu.so > $O/var.log 2>&1 || { echo "var failed"; tail -20 $O/var.log; exit 1; }
grep -v amdgpu.ids $O/var.log

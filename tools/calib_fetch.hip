// calib_fetch.hip — FETCH_SIZE calibration on gfx950 (MI355X_MICROARCH.md: "calibrate on a
// known byte count in your own access pattern"): streams a 1 GiB buffer once with 4, 8 and
// 16 bytes per lane, so rocprofv3 --pmc FETCH_SIZE can be compared with the exact bytes.
//   hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o gpurun_out/calib_fetch
#include <hip/hip_runtime.h>
#include <cstdio>

template <class T>
__global__ void stream_read(const T* __restrict__ x, size_t n, float* out) {
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = x[i];
    const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
    for (int q = 0; q < (int)(sizeof(T) / 4); ++q) acc += f[q];
  }
  if (acc == 12345.678f) out[0] = acc;  // keeps the loads alive
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  float* x = nullptr;
  float* out = nullptr;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(x, 0, bytes);
  const int grid = 256 * 8, block = 256;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream_read<float>, dim3(grid), dim3(block), 0, 0, x, bytes / 4, out);
    hipLaunchKernelGGL(stream_read<float2>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<float2*>(x), bytes / 8, out);
    hipLaunchKernelGGL(stream_read<float4>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<float4*>(x), bytes / 16, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("streamed %zu bytes per kernel\n", bytes);
  (void)hipFree(x);
  (void)hipFree(out);
  return 0;
}

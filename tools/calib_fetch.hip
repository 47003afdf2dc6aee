// calib_fetch.hip — FETCH_SIZE / WRITE_SIZE calibration on gfx950 (MI355X_MICROARCH.md:
// "calibrate on a known byte count in your own access pattern"): every kernel moves exactly
// 1 GiB once, so rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) per kernel divided by 1 GiB is the
// counter's scale for that access form.  The forms are the ones the engine's kernels use
// (tools/traffic.py names the calibration each kernel's traffic is corrected with):
//   stream_read<float|float2|float4>   4 / 8 / 16 B per lane, coalesced (trim_blocks: 16 B;
//                                      stft_mel / tuning_peaks on even offsets: 8 B)
//   pair_read                          two 4-byte loads per 8 bytes (stft_mel's odd-offset path)
//   lds_dma_read                       global_load_lds_dwordx4, 1 KiB per wave-instruction (the
//                                      CQT kernels' filter slices)
//   stream_write<float|float4>         4 / 16 B per lane (S_db rows / decimated octaves)
//   hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
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

// two dword loads per 8-byte element, as stft_mel reads a frame whose start is odd
__global__ void pair_read(const float* __restrict__ x, size_t n2, float* out) {
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const float* p = x + 2 * i;
    float a, b;
    asm volatile("global_load_dword %0, %2, off\n\tglobal_load_dword %1, %2, off offset:4\n\ts_waitcnt vmcnt(0)"
                 : "=&v"(a), "=&v"(b)
                 : "v"(p)
                 : "memory");
    acc += a + b;
  }
  if (acc == 12345.678f) out[0] = acc;
}

// LDS-DMA: each wave streams 1 KiB pieces into its own LDS slot (the CQT kernels' cm_dma16)
__global__ __launch_bounds__(256) void lds_dma_read(const uint4* __restrict__ x, size_t n16, float* out) {
  __shared__ uint4 slot[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)slot[wave];
  const size_t waves = (size_t)gridDim.x * 4;
  for (size_t piece = blockIdx.x * (size_t)4 + wave; piece * 64 < n16; piece += waves) {
    const uint4* p = x + piece * 64 + lane;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                 "s_waitcnt vmcnt(0)\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(p), "s"(__builtin_amdgcn_readfirstlane(base))
                 : "memory");
  }
  __syncthreads();
  if (slot[wave][lane].x == 0x12345678u) out[0] = 1.0f;
}

template <class T>
__global__ void stream_write(T* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v;
    float* f = reinterpret_cast<float*>(&v);
#pragma unroll
    for (int q = 0; q < (int)(sizeof(T) / 4); ++q) f[q] = (float)(i + q);
    y[i] = v;
  }
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  float* x = nullptr;
  float* y = nullptr;
  float* out = nullptr;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess)
    return 1;
  (void)hipMemset(x, 0, bytes);
  const int grid = 256 * 8, block = 256;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream_read<float>, dim3(grid), dim3(block), 0, 0, x, bytes / 4, out);
    hipLaunchKernelGGL(stream_read<float2>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<float2*>(x), bytes / 8, out);
    hipLaunchKernelGGL(stream_read<float4>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<float4*>(x), bytes / 16, out);
    hipLaunchKernelGGL(pair_read, dim3(grid), dim3(block), 0, 0, x, bytes / 8, out);
    hipLaunchKernelGGL(lds_dma_read, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const uint4*>(x), bytes / 16, out);
    hipLaunchKernelGGL(stream_write<float>, dim3(grid), dim3(block), 0, 0, y, bytes / 4);
    hipLaunchKernelGGL(stream_write<float4>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<float4*>(y), bytes / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("moved %zu bytes per kernel\n", bytes);
  (void)hipFree(x);
  (void)hipFree(y);
  (void)hipFree(out);
  return 0;
}

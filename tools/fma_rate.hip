// fma_rate.hip — measured VALU FMA throughput on this GPU for f32, packed f32 and f64
// (8 independent chains per lane, all CUs busy):
//   hipcc --offload-arch=gfx950 -O3 tools/fma_rate.hip -o tools/fma_rate && tools/fma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <class T>
__global__ __launch_bounds__(256) void chains(T* out, int iters, T a, T b) {
  T x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = (T)(threadIdx.x + i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = x[i] * a + b;  // contracted to one FMA
  }
  T s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == (T)12345.678) out[0] = s;
}

__global__ __launch_bounds__(256) void chains_pk(float2* out, int iters, float a, float b) {
  float2 x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = make_float2(threadIdx.x + i, threadIdx.x - i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      x[i].x = x[i].x * a + b;
      x[i].y = x[i].y * a + b;
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  if (s == 12345.678f) out[0] = make_float2(s, s);
}

template <class F>
double timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e-3;
}

int main() {
  int cu = 0;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cu * 16, block = 256, iters = 4096;
  void* out;
  hipMalloc(&out, 64);
  const double lanes = (double)grid * block;
  double t = timeit([&] { hipLaunchKernelGGL(chains<float>, dim3(grid), dim3(block), 0, 0, (float*)out, iters, 0.999f, 0.001f); });
  printf("f32 fma: %.1f TFLOP/s\n", lanes * iters * 8 * 2 / t / 1e12);
  t = timeit([&] { hipLaunchKernelGGL(chains_pk, dim3(grid), dim3(block), 0, 0, (float2*)out, iters, 0.999f, 0.001f); });
  printf("f32 fma (pairs): %.1f TFLOP/s\n", lanes * iters * 16 * 2 / t / 1e12);
  t = timeit([&] { hipLaunchKernelGGL(chains<double>, dim3(grid), dim3(block), 0, 0, (double*)out, iters, 0.999, 0.001); });
  printf("f64 fma: %.1f TFLOP/s\n", lanes * iters * 8 * 2 / t / 1e12);
  return 0;
}

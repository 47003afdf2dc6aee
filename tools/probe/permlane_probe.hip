// Prints where v_permlane32_swap / v_permlane16_swap move lanes (gfx950): A[l] = l, B[l] = 100 + l.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(l, 100u + l, false, false);
  auto s = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
  out[l] = r[0]; out[64 + l] = r[1]; out[128 + l] = s[0]; out[192 + l] = s[1];
}
int main() {
  unsigned* d; unsigned h[256];
  if (hipMalloc(&d, 1024) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char* nm[4] = {"p32 vdst", "p32 src ", "p16 vdst", "p16 src "};
  for (int t = 0; t < 4; ++t) { printf("%s:", nm[t]); for (int l = 0; l < 64; ++l) printf(" %u", h[64 * t + l]); printf("\n"); }
  return 0;
}

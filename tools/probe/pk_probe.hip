// Issue rate of packed f32 VALU (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32) against the
// scalar forms on gfx950: 8 independent chains per lane, many waves per SIMD, instruction
// throughput from hipEvent time.  Question: does a packed op (2 f32 results per lane) cost the
// issue slot of one scalar op, i.e. does packing halve the FFT butterflies' VALU time?
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
  float c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define F(n) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c##n) : "v"(a), "v"(b));
    REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

__global__ __launch_bounds__(256) void k_pkfma(float* out, float a, float b) {
  f2 av = {a, a}, bv = {b, b};
  f2 c0 = {(float)threadIdx.x, 1.f}, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6,
     c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define F(n) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c##n) : "v"(av), "v"(bv));
    REP8(F)
#undef F
  }
  f2 s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

__global__ __launch_bounds__(256) void k_add(float* out, float a, float b) {
  float c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define F(n) asm volatile("v_add_f32 %0, %1, %0" : "+v"(c##n) : "v"(a));
    REP8(F)
#undef F
  }
  out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

__global__ __launch_bounds__(256) void k_pkadd(float* out, float a, float b) {
  f2 av = {a, b};
  f2 c0 = {(float)threadIdx.x, 1.f}, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6,
     c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define F(n) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(c##n) : "v"(av));
    REP8(F)
#undef F
  }
  f2 s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

__global__ __launch_bounds__(256) void k_pkmul(float* out, float a, float b) {
  f2 av = {a, b};
  f2 c0 = {(float)threadIdx.x, 1.f}, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6,
     c7 = c0 + 7;
  for (int i = 0; i < ITERS; ++i) {
#define F(n) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(c##n) : "v"(av));
    REP8(F)
#undef F
  }
  f2 s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

// a mix as in a butterfly: one pk_add, one pk_add(neg), alternated with scalar fma
__global__ __launch_bounds__(256) void k_mix(float* out, float a, float b) {
  f2 av = {a, b};
  f2 c0 = {(float)threadIdx.x, 1.f}, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
  float d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3;
  for (int i = 0; i < ITERS; ++i) {
#define F(n) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(c##n) : "v"(av)); \
             asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(d##n) : "v"(a), "v"(b));
    F(0) F(1) F(2) F(3)
#undef F
  }
  f2 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + d0 + d1 + d2 + d3;
}

int main() {
  float* d;
  const int blocks = 256 * 8;  // 8 x 256-thread blocks per CU: 8 waves per SIMD
  if (hipMalloc(&d, sizeof(float) * blocks * 256) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct K {
    const char* name;
    void (*fn)(float*, float, float);
    double ops_per_instr;
  } ks[] = {{"v_fma_f32", k_fma, 1}, {"v_pk_fma_f32", k_pkfma, 2}, {"v_add_f32", k_add, 1},
            {"v_pk_add_f32", k_pkadd, 2}, {"v_pk_mul_f32", k_pkmul, 2}, {"mix pk_add+fma", k_mix, 1.5}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, d, 1.0001f, 0.9999f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr = (double)blocks * 4 /*waves*/ * ITERS * 8;  // wave-instructions
      if (rep == 2)
        printf("%-16s %.3f ms  %.1f wave-instr/ns  %.1f Tops/s (f32 results x lanes)\n", k.name, ms,
               instr / (ms * 1e6), instr * 64 * k.ops_per_instr / (ms * 1e9));
    }
  }
  return 0;
}

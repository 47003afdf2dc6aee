// vmcnt_order.hip — does `s_waitcnt vmcnt(N)` on gfx950 retire LDS-DMA
// (global_load_lds_dwordx4) and register loads (global_load_dwordx4) in issue order?
// (cqt_mfma_low_kernel's counted slice wait, csrc/cqt.hip c2_wait_slice.)
//
// Case A, the slice wait: one LDS-DMA piece from a cold line (HBM miss), then N register loads
// from hot lines (L2 hits), vmcnt(N), then the LDS piece is read.  If vmcnt counted the younger
// hot loads' completions first, the wait would be met with the DMA still in flight and the read
// would return the sentinel written before it.
// Case B, the round-5 block wait: one register load (a dword) from a cold line, then N LDS-DMA
// pieces from hot lines, vmcnt(N), then the register is copied inside the same asm block.  A register whose
// load had not landed still holds the sentinel.
// Every lane of every trial checks its 16 bytes; a fresh cold line per trial and lane group.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/vmcnt_order.hip -o tools/probe/vmcnt_order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr unsigned SENT = 0xdeadbeefu;
constexpr int TRIALS = 64;

__device__ __forceinline__ unsigned pattern(size_t i) { return (unsigned)(i * 2654435761u) ^ 0x5bd1e995u; }

__global__ void fill(uint4* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(pattern(4 * i), pattern(4 * i + 1), pattern(4 * i + 2), pattern(4 * i + 3));
}

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// case A: LDS-DMA (cold) then 4 register loads (hot), vmcnt(4), LDS read
__global__ __launch_bounds__(64) void case_a(const uint4* cold, const uint4* hot, size_t cold_n,
                                             unsigned long long* bad, unsigned long long* seen) {
  __shared__ uint4 slot[64];
  const int lane = threadIdx.x;
  unsigned long long nbad = 0;
  for (int t = 0; t < TRIALS; ++t) {
    slot[lane] = make_uint4(SENT, SENT, SENT, SENT);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    const size_t line = ((size_t)(t * gridDim.x + blockIdx.x) * 977 % (cold_n / 64)) * 64;
    const uint4* c = cold + line + lane;
    const uint4* h = hot + lane;
    uint4 r, t0, t1, t2, t3;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %[keep], m0\n\t"
        "s_mov_b32 m0, %[lds]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[c], off\n\t"
        "global_load_dwordx4 %[t0], %[h], off\n\t"
        "global_load_dwordx4 %[t1], %[h], off offset:1024\n\t"
        "global_load_dwordx4 %[t2], %[h], off offset:2048\n\t"
        "global_load_dwordx4 %[t3], %[h], off offset:3072\n\t"
        "s_waitcnt vmcnt(4)\n\t"
        "s_mov_b32 m0, %[keep]\n\t"
        "ds_read_b128 %[r], %[la]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_waitcnt vmcnt(0)"
        : [r] "=&v"(r), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [keep] "=&s"(keep)
        : [c] "v"(c), [h] "v"(h), [lds] "s"(__builtin_amdgcn_readfirstlane(lds_u32(slot))),
          [la] "v"(lds_u32(slot + lane))
        : "memory");
    const size_t i = line + lane;
    nbad += (r.x != pattern(4 * i)) | (r.y != pattern(4 * i + 1)) | (r.z != pattern(4 * i + 2)) |
            (r.w != pattern(4 * i + 3));
    if (t0.x == 12345u && t1.x == 12345u && t2.x == 12345u && t3.x == 12345u) nbad += 1000000;  // keep loads live
  }
  atomicAdd(bad, nbad);
  atomicAdd(seen, (unsigned long long)TRIALS);
}

// case B: register load (cold) then 4 LDS-DMA pieces (hot), vmcnt(4), register copy
__global__ __launch_bounds__(64) void case_b(const uint4* cold, const uint4* hot, size_t cold_n,
                                             unsigned long long* bad, unsigned long long* seen) {
  __shared__ uint4 ring[4 * 64];
  const int lane = threadIdx.x;
  unsigned long long nbad = 0;
  for (int t = 0; t < TRIALS; ++t) {
    const size_t line = ((size_t)(t * gridDim.x + blockIdx.x) * 1031 % (cold_n / 64)) * 64;
    const uint4* c = cold + line + lane;
    const uint4* h = hot + lane;
    unsigned r = SENT, o;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %[keep], m0\n\t"
        "global_load_dword %[r], %[c], off\n\t"
        "s_mov_b32 m0, %[l0]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[h], off\n\t"
        "s_mov_b32 m0, %[l1]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[h], off offset:1024\n\t"
        "s_mov_b32 m0, %[l2]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[h], off offset:2048\n\t"
        "s_mov_b32 m0, %[l3]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[h], off offset:3072\n\t"
        "s_waitcnt vmcnt(4)\n\t"
        "v_mov_b32 %[o], %[r]\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_mov_b32 m0, %[keep]"
        : [r] "+&v"(r), [o] "=&v"(o), [keep] "=&s"(keep)
        : [c] "v"(c), [h] "v"(h), [l0] "s"(__builtin_amdgcn_readfirstlane(lds_u32(ring))),
          [l1] "s"(__builtin_amdgcn_readfirstlane(lds_u32(ring + 64))),
          [l2] "s"(__builtin_amdgcn_readfirstlane(lds_u32(ring + 128))),
          [l3] "s"(__builtin_amdgcn_readfirstlane(lds_u32(ring + 192)))
        : "memory");
    const size_t i = line + lane;
    nbad += o != pattern(4 * i);
  }
  atomicAdd(bad, nbad);
  atomicAdd(seen, (unsigned long long)TRIALS);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
  const size_t cold_bytes = (size_t)2 << 30;  // 2 GiB: every trial line misses L2 and the 256 MB MALL
  const size_t cold_n = cold_bytes / sizeof(uint4);
  uint4 *cold, *hot;
  unsigned long long* cnt;
  CK(hipMalloc(&cold, cold_bytes));
  CK(hipMalloc(&hot, 64 * 1024));
  CK(hipMalloc(&cnt, 4 * sizeof(unsigned long long)));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, cold, cold_n);
  hipLaunchKernelGGL(fill, dim3(16), dim3(256), 0, 0, hot, (size_t)4096);
  CK(hipMemset(cnt, 0, 4 * sizeof(unsigned long long)));
  CK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r) {
    // a large evicting write between reps so the cold lines are cold again
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, cold, cold_n);
    hipLaunchKernelGGL(case_a, dim3(2048), dim3(64), 0, 0, cold, hot, cold_n, cnt + 0, cnt + 1);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, cold, cold_n);
    hipLaunchKernelGGL(case_b, dim3(2048), dim3(64), 0, 0, cold, hot, cold_n, cnt + 2, cnt + 3);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  unsigned long long h[4];
  CK(hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost));
  // every lane adds its own stale count and its TRIALS: both totals are per lane-trial
  std::printf("case A (LDS-DMA cold, then 4 register loads hot, vmcnt(4), read LDS): %llu stale of %llu lane-trials\n",
              h[0], h[1]);
  std::printf("case B (register load cold, then 4 LDS-DMA hot, vmcnt(4), read register): %llu stale of %llu lane-trials\n",
              h[2], h[3]);
  CK(hipFree(cold));
  CK(hipFree(hot));
  CK(hipFree(cnt));
  return 0;
}

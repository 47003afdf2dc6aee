// nc_block.h — workgroup-level primitives (LDS reductions, scans, radix select).
#pragma once
#include "nc_device.h"

namespace nc {

// Workgroup scratch for reductions: at least NT/64 * 16 bytes.
template <int NT>
struct BlockScratch {
  double d[NT / 64];
  long long l[NT / 64];
  int i[NT / 64];
};

template <int NT>
__device__ __forceinline__ double block_sum(double v, BlockScratch<NT>& s) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s.d[wave] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += s.d[i];
  return r;
}

template <int NT>
__device__ __forceinline__ double block_max(double v, BlockScratch<NT>& s) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s.d[wave] = v;
  __syncthreads();
  double r = s.d[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) r = fmax(r, s.d[i]);
  return r;
}

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int NT>
__device__ __forceinline__ int block_min_i(int v, BlockScratch<NT>& s) {
  v = wave_min_i(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s.i[wave] = v;
  __syncthreads();
  int r = s.i[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) r = min(r, s.i[i]);
  return r;
}
template <int NT>
__device__ __forceinline__ int block_max_i(int v, BlockScratch<NT>& s) {
  v = wave_max_i(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s.i[wave] = v;
  __syncthreads();
  int r = s.i[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) r = max(r, s.i[i]);
  return r;
}
template <int NT>
__device__ __forceinline__ int block_sum_i(int v, BlockScratch<NT>& s) {
  v = wave_sum_i(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s.i[wave] = v;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += s.i[i];
  return r;
}

// Exclusive prefix sum of one int per thread (in thread order) + total.
template <int NT>
__device__ __forceinline__ int block_exclusive_scan(int v, int& total, BlockScratch<NT>& s) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  __syncthreads();
  if (lane == 63) s.i[wave] = incl;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    if (i < wave) base += s.i[i];
    tot += s.i[i];
  }
  total = tot;
  return base + incl - v;
}

// Exclusive prefix sum of one int64 per thread (in thread order) + total; sh holds NT/64
// int64s of LDS.  Callers walk long lists in tiles of NT, carrying the total.
template <int NT>
__device__ __forceinline__ int64_t block_exclusive_scan64(int64_t v, int64_t& total, int64_t* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  __syncthreads();
  if (lane == 63) sh[wave] = incl;
  __syncthreads();
  int64_t base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    if (i < wave) base += sh[i];
    tot += sh[i];
  }
  total = tot;
  return base + incl - v;
}

// base[i] = sum_{q<i} count(q) for i in [0, n], one workgroup of NT threads (a parallel
// replacement of a one-thread prefix loop over files / chunks).
template <int NT, typename F>
__device__ __forceinline__ void block_prefix_table(int n, int64_t* base, F count) {
  __shared__ int64_t sh[NT / 64];
  int64_t carry = 0;
  for (int t0 = 0; t0 < n; t0 += NT) {
    const int i = t0 + (int)threadIdx.x;
    const int64_t v = i < n ? count(i) : 0;
    int64_t tot = 0;
    const int64_t ex = block_exclusive_scan64<NT>(v, tot, sh);
    if (i < n) base[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) base[n] = carry;
}

// (value, index) argmax with numpy semantics: NaN wins, ties -> smallest index.
__device__ __forceinline__ bool np_better(double a, int ia, double b, int ib) {
  const bool na = a != a, nb = b != b;
  if (na || nb) {
    if (na && nb) return ia < ib;
    return na;
  }
  if (a > b) return true;
  if (a < b) return false;
  return ia < ib;
}
// numpy-order argmax over the wave, the result in every lane: DPP quad swaps, half-row and
// row mirrors, row broadcasts into the odd / upper rows (lanes outside a row mask see the
// identity (-inf, INT_MAX)), then lane 63's pair.  np_better is a total order, so the
// reduction order does not change the result.
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
  const long long idb = __double_as_longlong(-INFINITY);
  auto step = [&](auto ctrl, auto rmask) {
    constexpr int C = decltype(ctrl)::value, M = decltype(rmask)::value;
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<C, M>((int)(unsigned)b, (int)(unsigned)idb);
    const int hi = dpp_i<C, M>((int)(unsigned)(b >> 32), (int)(unsigned)(idb >> 32));
    const int oi = dpp_i<C, M>(i, 0x7fffffff);
    const double ov = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
    if (np_better(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  };
  step(std::integral_constant<int, 0xB1>{}, std::integral_constant<int, 0xf>{});
  step(std::integral_constant<int, 0x4E>{}, std::integral_constant<int, 0xf>{});
  step(std::integral_constant<int, 0x141>{}, std::integral_constant<int, 0xf>{});
  step(std::integral_constant<int, 0x140>{}, std::integral_constant<int, 0xf>{});
  step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xa>{});
  step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xc>{});
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), 63);
  v = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
  i = __builtin_amdgcn_readlane(i, 63);
}
template <int NT>
__device__ __forceinline__ void block_argmax(double& v, int& i, BlockScratch<NT>& s) {
  wave_argmax(v, i);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    s.d[wave] = v;
    s.i[wave] = i;
  }
  __syncthreads();
  v = s.d[0];
  i = s.i[0];
#pragma unroll
  for (int k = 1; k < NT / 64; ++k)
    if (np_better(s.d[k], s.i[k], v, i)) {
      v = s.d[k];
      i = s.i[k];
    }
}

__device__ __forceinline__ unsigned long long dkey(double x) {
  unsigned long long u = (unsigned long long)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dunkey(unsigned long long k) {
  const unsigned long long u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}

// k-th smallest (0-based) of vals[i] over i in [0,n) with flag[i] != 0.
// 8 passes of 8-bit radix select; hist = 256 ints of LDS.
template <int NT>
__device__ double block_kth_flagged(const double* vals, const uint8_t* flag, int n, int k, int* hist,
                                    BlockScratch<NT>& s) {
  unsigned long long prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += NT) {
      if (!flag[i]) continue;
      const unsigned long long key = dkey(vals[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // digit pick: 4 bins per lane + a wave prefix scan (no serial walk)
      const int lane = threadIdx.x;
      const int h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
      const int sum = h0 + h1 + h2 + h3;
      int incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      const int excl = incl - sum;
      if (excl <= k && k < incl) {
        int r = k - excl, d = 4 * lane;
        if (r >= h0) {
          r -= h0;
          ++d;
          if (r >= h1) {
            r -= h1;
            ++d;
            if (r >= h2) {
              r -= h2;
              ++d;
            }
          }
        }
        s.l[0] = (long long)d;
        s.i[0] = r;
      }
    }
    __syncthreads();
    const unsigned long long d = (unsigned long long)s.l[0];
    k = s.i[0];
    prefix |= d << shift;
    mask |= 255ull << shift;
    __syncthreads();
  }
  return dunkey(prefix);
}

}  // namespace nc

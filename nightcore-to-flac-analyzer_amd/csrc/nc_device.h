// nc_device.h — shared CDNA4 (gfx950) device helpers for the nightcore engine.
//
// * complex float2 arithmetic
// * wave64 reductions (shuffle based; wave = 64 lanes on CDNA, never 32)
// * a one-wave Stockham auto-sort FFT (mixed radix 4/8/16) working on an LDS
//   buffer with a 1-in-16 pad (bank-conflict break for the stride-R writes of
//   the first stage), inputs of stage 1 taken straight from registers.
//
// Every FFT here is forward (e^{-2 pi i nk/N}); inverses use the conjugation
// identity.  Twiddles come from an 8192-entry table built on the host in double
// precision (exp(-2 pi i m / 8192) rounded to f32), so one table serves all
// complex N <= 4096 (real 8192).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nc_span.h"

#define NC_WAVE 64

namespace nc {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// multiply by -i
__device__ __forceinline__ float2 cmul_mi(float2 a) { return make_float2(a.y, -a.x); }

// 10 * log10f(fmaxf(1e-10f, x)) bit for bit (librosa power_to_db's floor, amin = 1e-10): the
// floored argument is a normal float, so log10f's denormal rescale (v_ldexp, two selects and the
// subtract of its offset) is dropped; what stays is its own sequence, v_log_f32 and the product
// with log10(2) compensated in f32 (ch + cl), and its non-finite select.  9 VALU against 14.
#ifndef NC_DB_LIB_
#define NC_DB_LIB_ 0  // A/B probe: the library log10f instead
#endif
__device__ __forceinline__ float db10_floor(float x) {
  if (NC_DB_LIB_) return 10.0f * log10f(fmaxf(1e-10f, x));
  const float l = __builtin_amdgcn_logf(fmaxf(1e-10f, x));
  const float ch = __uint_as_float(0x3e9a209au), cl = __uint_as_float(0x3284fbcfu);
  const float ph = __fmul_rn(l, ch);
  float e = __builtin_fmaf(l, ch, -ph);
  e = __builtin_fmaf(l, cl, e);
  const float r = __builtin_fmaf(ch, l, e);
  return 10.0f * (__builtin_fabsf(l) < __builtin_inff() ? r : l);
}

// ------------------------------------------------------------------ workgroup frame queue
// A persistent workgroup's frames handed to its waves one at a time from an LDS counter (round 6):
// the frames in flight are always the ones taken last, whatever the waves' relative speeds, so
// neighbouring frames (which share 3/4 of their samples) meet in L1 / L2 together, and no wave
// idles at the end while another still holds a static share.  A static interleave (wave w: frames
// 16 G + w) let the waves drift tens of groups apart: stft_mel read 1.62x its algorithmic bytes
// and ran 9.8 % slower.  Each wave reserves its next frame when it starts one, so the atomic's
// latency hides under the frame.  `ctr` is zeroed before the workgroup barrier that precedes the
// first take; frames come out increasing per wave (the descriptor tracking relies on it).
struct WgFrameQueue {
  int* ctr;
  int nx;  // lane 0: the reserved frame
  __device__ __forceinline__ int reserve(int lane) {
    int r = 0;
    if (lane == 0) r = atomicAdd(ctr, 1);
    return r;
  }
  __device__ __forceinline__ WgFrameQueue(int* c, int lane) : ctr(c) { nx = reserve(lane); }
  // the next frame index of this workgroup's range (>= its frame count: done)
  __device__ __forceinline__ int take(int lane) {
    const int n = __builtin_amdgcn_readfirstlane(nx);
    nx = reserve(lane);
    return n;
  }
};

// ------------------------------------------------------------------ wave reductions
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// DPP reductions whose result is wave-uniform (read from lane 63 into an SGPR): quad
// swaps, half-row and row mirrors, then row_bcast15 / row_bcast31 into the odd / upper
// rows -- VALU ops with a DPP source instead of the LDS-crossbar ds_bpermute of __shfl_xor.
// Lanes outside a row mask take `old` (the operation's identity).  Fixed order, so
// deterministic; the order differs from wave_sum's butterfly.
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ int dpp_i(int v, int old) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xf, false);
}
// v + v of the DPP source lane CTRL (every lane of every row; a partner outside the row pattern
// is not used by the controls passed here: quad perms and row mirrors)
template <int CTRL>
__device__ __forceinline__ double dpp_add_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_i<CTRL, 0xf>((int)(unsigned)b, 0), hi = dpp_i<CTRL, 0xf>((int)(unsigned)(b >> 32), 0);
  return v + __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <class Op>
__device__ __forceinline__ float wave_reduce_u(float v, float id, Op op) {
  auto step = [&](auto ctrl, auto rmask) {
    constexpr int C = decltype(ctrl)::value, M = decltype(rmask)::value;
    v = op(v, __int_as_float(dpp_i<C, M>(__float_as_int(v), __float_as_int(id))));
  };
  step(std::integral_constant<int, 0xB1>{}, std::integral_constant<int, 0xf>{});   // quad_perm [1,0,3,2]
  step(std::integral_constant<int, 0x4E>{}, std::integral_constant<int, 0xf>{});   // quad_perm [2,3,0,1]
  step(std::integral_constant<int, 0x141>{}, std::integral_constant<int, 0xf>{});  // row_half_mirror
  step(std::integral_constant<int, 0x140>{}, std::integral_constant<int, 0xf>{});  // row_mirror
  step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xa>{});  // row_bcast15
  step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xc>{});  // row_bcast31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_max_u(float v) {
  return wave_reduce_u(v, -INFINITY, [](float x, float y) { return fmaxf(x, y); });
}
__device__ __forceinline__ double wave_sum_u(double v) {
  auto step = [&](auto ctrl, auto rmask) {
    constexpr int C = decltype(ctrl)::value, M = decltype(rmask)::value;
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<C, M>((int)(unsigned)b, 0), hi = dpp_i<C, M>((int)(unsigned)(b >> 32), 0);
    v += __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
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
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ------------------------------------------------------------------ kernel spans (nc_profile)
// A profiled launch gets kSpanLines (start, end) slots, one 128-byte line each (start init
// ~0, end init 0).  The first kSpanEdge workgroups of the grid lower a start (thread 0),
// the last kSpanEdge raise an end (lane 0 of every wave) on the 100 MHz wall clock (both
// recorded at exit, the start as read at entry), each
// in line (linear workgroup id mod kSpanLines): min start .. max end is the kernel's
// execution span, the duration rocprofv3 --kernel-trace reports, unaffected by queueing
// behind other streams' kernels.  Device-scope atomics on one address serialise (tens of
// ns each), hence the lines and the edge-only recording: a launch issues at most
// 2 kSpanEdge x waves atomics, <= kSpanEdge / kSpanLines x waves per line.  Fire-and-forget;
// null = not profiled.
__device__ __forceinline__ unsigned span_lin() {
  return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}
__device__ __forceinline__ void span_record(unsigned long long* sp, unsigned long long t0) {
  if (sp && (threadIdx.x & 63) == 0) {
    const unsigned n = gridDim.x * gridDim.y * gridDim.z, l = span_lin();
    unsigned long long* line = sp + (l % kSpanLines) * kSpanStride;
    if (threadIdx.x == 0 && l < (unsigned)kSpanEdge) atomicMin(line, t0);
    if (l + (unsigned)kSpanEdge >= n) atomicMax(line + 1, (unsigned long long)wall_clock64());
  }
}

// RAII form for a kernel body: the start time is read at construction (a wave-uniform
// value in SGPRs) and both records are made at every exit of the scope, so the kernel
// prologue has no divergent branch (a lane-0 atomic at entry cost cqt_chroma 13 VGPRs
// and its spill-free allocation, decimate3 one wave per SIMD)
struct Span {
  unsigned long long* sp;
  unsigned long long t0;
  __device__ __forceinline__ explicit Span(unsigned long long* p) : sp(p), t0(p ? wall_clock64() : 0ull) {}
  __device__ __forceinline__ ~Span() { span_record(sp, t0); }
};

// XCD-aware workgroup order (cdna_hip_programming.md T1): the dispatcher deals linear
// workgroup ids round robin to the 8 XCDs (blockIdx % 8 labels the workgroups that share an
// L2); this bijective remap gives each of those classes a contiguous 1/8 of the logical ids, so
// neighbouring logical work (the same chunk, the same tuning's filters) shares one L2.  Speed
// only: any placement computes the same results.
__device__ __forceinline__ unsigned xcd_remap(unsigned l, unsigned n) {
  const unsigned q = n / 8, r = n % 8, x = l % 8;
  return x * q + min(x, r) + l / 8;
}

// float <-> order-preserving int (for atomicMax on floats of either sign)
__device__ __forceinline__ int f2ord(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

// ------------------------------------------------------------------ in-register DFTs
// exp(-2 pi i m / 16) for the odd m (compile-time after unrolling)
__device__ __forceinline__ float2 w16(int m) {
  switch (m) {
    case 1: return make_float2(9.238795325e-01f, -3.826834324e-01f);
    case 3: return make_float2(3.826834324e-01f, -9.238795325e-01f);
    case 5: return make_float2(-3.826834324e-01f, -9.238795325e-01f);
    default: return make_float2(-9.238795325e-01f, -3.826834324e-01f);  // 7
  }
}

// twiddle exp(-2 pi i k / R) * o with k, R compile-time after unrolling (k < R/2)
template <int R>
__device__ __forceinline__ float2 twr(int k, float2 o) {
  const int m = k * (16 / R);
  if (m == 0) return o;
  if (m == 4) return cmul_mi(o);
  const float s = 7.071067812e-01f;
  if (m == 2) return make_float2(s * (o.x + o.y), s * (o.y - o.x));   // (s, -s)
  if (m == 6) return make_float2(s * (o.y - o.x), -s * (o.x + o.y));  // (-s, -s)
  return cmul(w16(m), o);
}

template <int R>
struct DFT {
  static __device__ __forceinline__ void run(float2* v) {
    float2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    DFT<R / 2>::run(e);
    DFT<R / 2>::run(o);
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const float2 t = twr<R>(k, o[k]);
      v[k] = cadd(e[k], t);
      v[k + R / 2] = csub(e[k], t);
    }
  }
};
template <>
struct DFT<1> {
  static __device__ __forceinline__ void run(float2*) {}
};
template <>
struct DFT<2> {
  static __device__ __forceinline__ void run(float2* v) {
    const float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  }
};
template <>
struct DFT<4> {
  static __device__ __forceinline__ void run(float2* v) {
    const float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
    const float2 s13 = cadd(v[1], v[3]), d13 = cmul_mi(csub(v[1], v[3]));
    v[0] = cadd(s02, s13);
    v[2] = csub(s02, s13);
    v[1] = cadd(d02, d13);
    v[3] = csub(d02, d13);
  }
};

// Wave-uniform values the compiler cannot prove uniform (derived from the wave id or
// from loads indexed by it): pin them to SGPRs so addressing stays scalar.
__device__ __forceinline__ int uniform32(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// ------------------------------------------------------------------ Stockham wave FFT
// Exchange layout of the 1024-point wave FFT: one pad element per 32.  ds_read_b64 services
// 32 lanes over all 64 banks, so the stage-2 reads (element l + 64 r) need 32 consecutive
// elements on distinct banks, which a pad every 16 breaks (lanes 0 and 31 collide: 2x on every
// read).  The stage-1 writes (element 16 j + r, 16-lane groups on 32 banks) stay conflict free
// when lane l takes j = fft_in_lane(l) (below) instead of j = l.
__device__ __forceinline__ int lpad(int i) { return i + (i >> 5); }
// Stage-1 butterfly of lane l: j = 2 (l mod 16) + bit 4 of l, + 32 for the upper half-wave, so
// the 16 lanes of a ds_write_b64 group write rows j whose pads j / 2 differ.  The input reads
// x[j + 64 r] stay one contiguous 512-byte span per load.
__device__ __forceinline__ int fft_in_lane(int l) { return (((l & 15) << 1) | ((l >> 4) & 1)) | (l & 32); }

// f(std::integral_constant<int, i>{}) for i < N_, unrolled by construction: the loop unroller
// leaves loops around inline asm alone, and a rolled loop over a register array homes the
// array in scratch
template <int I, int N_, class F>
__device__ __forceinline__ void static_for_impl(F&& f) {
  if constexpr (I < N_) {
    f(std::integral_constant<int, I>{});
    static_for_impl<I + 1, N_>(f);
  }
}
template <int N_, class F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl<0, N_>(f); }

// LDS reads issued as one batch of ds_read_b64 and one wait.  The compiler pairs neighbouring
// 8-byte LDS reads into ds_read2_b64 / ds_read2st64_b64, which cost 8 LDS cycles where two
// ds_read_b64 cost 2 + 2 (MI355X_MICROARCH.md, LDS table); for the FFT exchanges that is a
// fifth of the kernels' LDS time.  An asm block is never merged; its outputs are defined
// only after its own s_waitcnt, so no consumer can see a pending register.
typedef float nc_f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)p;  // generic LDS pointer: aperture | offset
}
#define NC_RD_(i, a, o) "ds_read_b64 %" #i ", %" #a " offset:%" #o "\n\t"
// o[i] = *(float2*)(a[i / 4] + off[i]), i < 16: four base addresses, 16 byte offsets
template <int O0, int O1, int O2, int O3, int O4, int O5, int O6, int O7, int O8, int O9, int O10, int O11,
          int O12, int O13, int O14, int O15>
__device__ __forceinline__ void lds_read16(float2 (&o)[16], uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  // separate scalars, not an array: asm outputs into an array are homed in scratch
  nc_f2v d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15;
  asm volatile(NC_RD_(0, 16, 20) NC_RD_(1, 16, 21) NC_RD_(2, 16, 22) NC_RD_(3, 16, 23)
               NC_RD_(4, 17, 24) NC_RD_(5, 17, 25) NC_RD_(6, 17, 26) NC_RD_(7, 17, 27)
               NC_RD_(8, 18, 28) NC_RD_(9, 18, 29) NC_RD_(10, 18, 30) NC_RD_(11, 18, 31)
               NC_RD_(12, 19, 32) NC_RD_(13, 19, 33) NC_RD_(14, 19, 34) NC_RD_(15, 19, 35)
               "s_waitcnt lgkmcnt(0)"
               : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(d4), "=&v"(d5), "=&v"(d6), "=&v"(d7),
                 "=&v"(d8), "=&v"(d9), "=&v"(d10), "=&v"(d11), "=&v"(d12), "=&v"(d13), "=&v"(d14), "=&v"(d15)
               : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "i"(O0), "i"(O1), "i"(O2), "i"(O3), "i"(O4), "i"(O5),
                 "i"(O6), "i"(O7), "i"(O8), "i"(O9), "i"(O10), "i"(O11), "i"(O12), "i"(O13), "i"(O14), "i"(O15)
               : "memory");
  o[0] = make_float2(d0.x, d0.y);
  o[1] = make_float2(d1.x, d1.y);
  o[2] = make_float2(d2.x, d2.y);
  o[3] = make_float2(d3.x, d3.y);
  o[4] = make_float2(d4.x, d4.y);
  o[5] = make_float2(d5.x, d5.y);
  o[6] = make_float2(d6.x, d6.y);
  o[7] = make_float2(d7.x, d7.y);
  o[8] = make_float2(d8.x, d8.y);
  o[9] = make_float2(d9.x, d9.y);
  o[10] = make_float2(d10.x, d10.y);
  o[11] = make_float2(d11.x, d11.y);
  o[12] = make_float2(d12.x, d12.y);
  o[13] = make_float2(d13.x, d13.y);
  o[14] = make_float2(d14.x, d14.y);
  o[15] = make_float2(d15.x, d15.y);
}
// o[i] = *(float2*)(a[i] + O[i]), i < 3 (twiddle batches)
template <int O0, int O1, int O2>
__device__ __forceinline__ void lds_read3(float2 (&o)[3], uint32_t a0, uint32_t a1, uint32_t a2) {
  nc_f2v d0, d1, d2;
  asm volatile(NC_RD_(0, 3, 6) NC_RD_(1, 4, 7) NC_RD_(2, 5, 8) "s_waitcnt lgkmcnt(0)"
               : "=&v"(d0), "=&v"(d1), "=&v"(d2)
               : "v"(a0), "v"(a1), "v"(a2), "i"(O0), "i"(O1), "i"(O2)
               : "memory");
  o[0] = make_float2(d0.x, d0.y);
  o[1] = make_float2(d1.x, d1.y);
  o[2] = make_float2(d2.x, d2.y);
}
// v[i] *= twiddle row ROW + i (rows S bytes apart from a), i < 3
template <int ROW, int S>
__device__ __forceinline__ void tw_batch3(float2* v, uint32_t a) {
  float2 w[3];
  lds_read3<ROW * S, (ROW + 1) * S, (ROW + 2) * S>(w, a, a, a);
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] = cmul(v[i], w[i]);
}
// 16 reads from one base at byte offsets O + i S
template <int O, int S>
__device__ __forceinline__ void lds_read16_strided(float2 (&o)[16], uint32_t a) {
  lds_read16<O, O + S, O + 2 * S, O + 3 * S, O + 4 * S, O + 5 * S, O + 6 * S, O + 7 * S, O + 8 * S, O + 9 * S,
             O + 10 * S, O + 11 * S, O + 12 * S, O + 13 * S, O + 14 * S, O + 15 * S>(o, a, a, a, a);
}
template <int N>
struct LdsSize {
  static constexpr int value = N + N / 32;  // float2 elements
};

// Stage with radix R, NS = product of the previous radices, NT threads (lanes of
// one wave when NT == 64, a whole workgroup otherwise; SYNC adds the barriers a
// multi-wave in-place stage needs).  Stage-1 input comes from registers in the
// layout x[j + r*N/R], j = tid + NT*b.
// Twiddles: TWN > 0 reads tw[q] = exp(-2 pi i q / TWN) (the 8192-entry global table or a
// copy); TWN == 0 reads a per-stage table laid out [r - 1][k] starting at STO (see
// StagedTw), whose reads are contiguous in k and so free of LDS bank conflicts.
template <int N, int R, int NS, int NT, bool SYNC, int TWN = 8192, int STO = 0>
__device__ __forceinline__ void stockham_stage_regs(float2 (&v)[N / (R * NT)][R], float2* lds,
                                                    const float2* __restrict__ tw, int tid) {
  constexpr int NB = N / (R * NT);
  static_assert(NB >= 1, "radix too large for the thread count");
  static_assert(NS == 1 || NS == 16 || NS % 32 == 0, "stride offsets assume the pad-per-32 layout");
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = tid + NT * b;
    const int k = j % NS;
    if constexpr (NS > 1 && TWN == 0 && R == 16) {
      // 15 twiddles from the LDS table in five batches of three ds_read_b64
      const uint32_t ta = lds_addr(tw + STO + k);
      tw_batch3<0, NS * 8>(v[b] + 1, ta);
      tw_batch3<3, NS * 8>(v[b] + 4, ta);
      tw_batch3<6, NS * 8>(v[b] + 7, ta);
      tw_batch3<9, NS * 8>(v[b] + 10, ta);
      tw_batch3<12, NS * 8>(v[b] + 13, ta);
    } else if (NS > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r)
        v[b][r] = cmul(v[b][r], TWN > 0 ? tw[(k * r * (TWN > 0 ? TWN / (NS * R) : 1)) & (TWN - 1)]
                                        : tw[STO + (r - 1) * NS + k]);
    }
    DFT<R>::run(v[b]);
  }
  if (SYNC) __syncthreads();  // every thread has loaded this stage's inputs
  // lpad(base + r NS) == lpad(base) + lpad(r NS) when NS % 32 == 0, or NS == 16 (base % 32 is
  // then k < 16), so the strides become immediate LDS offsets instead of per-access index math
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int j = tid + NT * b;
    const int k = j % NS;
    const int base = (j / NS) * NS * R + k;
    if constexpr (NS % 16 == 0) {
      float2* p = lds + lpad(base);
#pragma unroll
      for (int r = 0; r < R; ++r) p[lpad(r * NS)] = v[b][r];
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) lds[lpad(base + r * NS)] = v[b][r];
    }
  }
  if (SYNC) __syncthreads();
}

template <int N, int R, int NS, int NT, bool SYNC, int TWN = 8192, int STO = 0>
__device__ __forceinline__ void stockham_stage(float2* lds, const float2* __restrict__ tw, int tid) {
  constexpr int NB = N / (R * NT);
  float2 v[NB][R];
  if constexpr (NT % 32 == 0 && (N / R) % 32 == 0) {
    const float2* p = lds + lpad(tid);
    if constexpr (NB == 1 && R == 16) {
      lds_read16_strided<0, (N / R) * 33 / 32 * 8>(v[0], lds_addr(p));
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < R; ++r) v[b][r] = p[lpad(NT * b + r * (N / R))];
    }
  } else {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int j = tid + NT * b;
#pragma unroll
      for (int r = 0; r < R; ++r) v[b][r] = lds[lpad(j + r * (N / R))];
    }
  }
  stockham_stage_regs<N, R, NS, NT, SYNC, TWN, STO>(v, lds, tw, tid);
}

// Radix plans: 512 = 8.8.8, 1024 = 16.16.4, 2048 = 16.16.8, 4096 = 16.16.16
template <int N>
struct Plan;
template <>
struct Plan<512> {
  static constexpr int R0 = 8, R1 = 8, R2 = 8;
};
template <>
struct Plan<1024> {
  static constexpr int R0 = 16, R1 = 16, R2 = 4;
};
template <>
struct Plan<2048> {
  static constexpr int R0 = 16, R1 = 16, R2 = 8;
};
template <>
struct Plan<4096> {
  static constexpr int R0 = 16, R1 = 16, R2 = 16;
};

// Stage-1 input register image: in[b][r] = x[(tid + NT b) + r * N / R0].
template <int N, int NT = 64>
using FftIn = float2[N / (Plan<N>::R0 * NT)][Plan<N>::R0];

template <int N, int NT, bool SYNC, int TWN = 8192>
__device__ __forceinline__ void fft_impl(FftIn<N, NT>& in, float2* lds, const float2* __restrict__ tw, int tid) {
  constexpr int R0 = Plan<N>::R0, R1 = Plan<N>::R1, R2 = Plan<N>::R2;
  static_assert(R0 * R1 * R2 == N, "plan");
  static_assert(TWN == 0 || TWN >= N, "twiddle table too coarse for this FFT");
  stockham_stage_regs<N, R0, 1, NT, SYNC, TWN, 0>(in, lds, tw, tid);
  stockham_stage<N, R1, R0, NT, SYNC, TWN, 0>(lds, tw, tid);
  stockham_stage<N, R2, R0 * R1, NT, SYNC, TWN, (R1 - 1) * R0>(lds, tw, tid);
}

// Per-stage twiddle table of an N-point complex FFT (+ the real-split twiddles of
// the 2N-point real transform), for TWN == 0:
//   [0, s3)          stage 2: W_{R0 R1}^{k r}  at (r - 1) R0 + k
//   [s3, split)      stage 3: W_N^{k r}        at s3 + (r - 1) R0 R1 + k
//   [split, size)    split:   W_{2N}^{k}       at split + k, k <= N/2
template <int N>
struct StagedTw {
  static constexpr int R0 = Plan<N>::R0, R1 = Plan<N>::R1, R2 = Plan<N>::R2;
  static constexpr int s3 = (R1 - 1) * R0;
  static constexpr int split = s3 + (R2 - 1) * R0 * R1;
  static constexpr int size = split + N / 2 + 1;
};

// Fill the staged table from the global 8192-entry table (all threads of a workgroup).
template <int N>
__device__ __forceinline__ void fill_staged_tw(float2* dst, const float2* __restrict__ tw8192, int tid, int nt) {
  using S = StagedTw<N>;
  for (int i = tid; i < S::size; i += nt) {
    int q;
    if (i < S::s3) {
      const int r = i / S::R0 + 1, k = i % S::R0;
      q = k * r * (8192 / (S::R0 * S::R1));
    } else if (i < S::split) {
      const int ii = i - S::s3, r = ii / (S::R0 * S::R1) + 1, k = ii % (S::R0 * S::R1);
      q = k * r * (8192 / N);
    } else {
      q = (i - S::split) * (8192 / (2 * N));
    }
    dst[i] = tw8192[q & 8191];
  }
}

// One wave; no barrier needed (LDS ops of a wave complete in order and every
// stage loads all of its inputs before its first store).  Natural-order output
// in lds (padded indexing).
// TWN is the length of the twiddle table tw[q] = exp(-2 pi i q / TWN): the
// 8192-entry global table, or a smaller copy staged in LDS.
template <int N, int TWN = 8192>
__device__ __forceinline__ void wave_fft(FftIn<N, 64>& in, float2* lds, const float2* __restrict__ tw, int lane) {
  fft_impl<N, 64, false, TWN>(in, lds, tw, lane);
}

// Whole workgroup of NT threads (all must call); output valid after return.
template <int N, int NT>
__device__ __forceinline__ void block_fft(FftIn<N, NT>& in, float2* lds, const float2* __restrict__ tw, int tid) {
  fft_impl<N, NT, true>(in, lds, tw, tid);
}

// ------------------------------------------------------------------ mirror-paired last stage
// Last radix-4 stage (NS = 256) of the 1024-point plan 16.16.4 done on the lane's butterfly
// set J = {l, 128-l, 128+l, 256-l} (lane 0: {0, 64, 192, 128}) instead of j = l + 64 b.  The
// set is closed under j -> 256 - j, so every output Z[k] sits in the same lane as its mirror
// Z[1024 - k]: real-input splits need neither a final LDS write nor a cross-lane read.
// v[b][r] = Z[J_b + 256 r].  STW3 = offset of the stage-3 table W_1024^{j r} at [r - 1][j].
__device__ __forceinline__ int mirror_J(int l, int b) {
  return b == 0 ? l : b == 1 ? (l ? 128 - l : 64) : b == 2 ? (l ? 128 + l : 192) : (l ? 256 - l : 128);
}

// TWB batches the stage twiddle reads too (asm); a kernel with little register headroom
// (spectral_frames) keeps them compiler-scheduled, or the compiler homes v in scratch.
template <int STW3, bool TWB = false>
__device__ __forceinline__ void fft1024_last_mirror(const float2* lds, const float2* tw, int l, float2 (&v)[4][4]) {
  // lpad(J + 256 r) = lpad(J) + 264 r: four bases, immediate offsets
  float2 o[16];
  lds_read16<0, 2112, 4224, 6336, 0, 2112, 4224, 6336, 0, 2112, 4224, 6336, 0, 2112, 4224, 6336>(
      o, lds_addr(lds + lpad(mirror_J(l, 0))), lds_addr(lds + lpad(mirror_J(l, 1))),
      lds_addr(lds + lpad(mirror_J(l, 2))), lds_addr(lds + lpad(mirror_J(l, 3))));
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[b][r] = o[4 * b + r];
  if constexpr (TWB) {
    static_for<4>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      float2 w[3];
      const uint32_t a = lds_addr(tw + STW3 + mirror_J(l, b));
      lds_read3<0, 2048, 4096>(w, a, a, a);
#pragma unroll
      for (int r = 1; r < 4; ++r) v[b][r] = cmul(v[b][r], w[r - 1]);
      DFT<4>::run(v[b]);
    });
  } else {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int r = 1; r < 4; ++r) v[b][r] = cmul(v[b][r], tw[STW3 + (r - 1) * 256 + mirror_J(l, b)]);
      DFT<4>::run(v[b]);
    }
  }
}

// Real-FFT split of a 2048-sample real frame packed as z[n] = x[2n] + i x[2n+1] from the
// mirror-paired outputs: f(k, X[k], X[1024 - k]) for the lane's 8 pairs (9 on lane 0),
// k <= 512, together covering X[0..1024] once (X[512] twice on lane 0).  SPLIT = offset of
// W_2048^k in tw.
// HALF = false: the outputs are 2 X[k] exactly (the two 0.5 scalings left out: a power-of-two
// scale commutes with every rounding of the split, so |2X|^2 = 4 |X|^2 bit for bit); callers
// that only compare or project |X|^2 fold the factor into their constants.
template <int SPLIT, bool HALF = true, bool OPAQUE0 = false, class F>
__device__ __forceinline__ void rsplit_mirror(const float2 (&v)[4][4], const float2* tw, int l, F&& f) {
  const bool l0 = l == 0;
  const int J1 = l0 ? 64 : 128 - l, J2 = l0 ? 192 : 128 + l, J3 = l0 ? 128 : 256 - l;
  auto pair = [&](float2 za, float2 zm, int k) {
    const float2 b = cconj(zm);
    const float2 E = HALF ? cscale(cadd(za, b), 0.5f) : cadd(za, b);
    const float2 O = cmul_mi(HALF ? cscale(csub(za, b), 0.5f) : csub(za, b));  // (a-b)/(2i), or 2x
    const float2 WO = cmul(tw[SPLIT + k], O);
    f(k, cadd(E, WO), cconj(csub(E, WO)));
  };
  // OPAQUE0: lane 0's operands as opaque values. A select between two elements of v can be
  // folded into a load through a selected address, which puts v in scratch (spectral_frames:
  // 10 scratch accesses per frame); where it is not (stft_mel, tuning_peaks) the barrier only
  // costs moves
  auto sel = [&](float2 a, float2 b) {
    if constexpr (OPAQUE0) asm("" : "+v"(a.x), "+v"(a.y));
    return make_float2(l0 ? a.x : b.x, l0 ? a.y : b.y);
  };
  pair(v[0][0], sel(v[0][0], v[3][3]), l);
  pair(v[0][1], sel(v[0][3], v[3][2]), l + 256);
  pair(sel(v[0][2], v[3][1]), v[0][2], l0 ? 512 : J3 + 256);
  pair(v[3][0], sel(v[3][3], v[0][3]), J3);
  pair(v[1][0], v[2][3], J1);
  pair(v[1][1], v[2][2], J1 + 256);
  pair(v[2][1], v[1][2], J2 + 256);
  pair(v[2][0], v[1][3], J2);
  if (l0) pair(v[3][1], v[3][2], 384);
}

}  // namespace nc

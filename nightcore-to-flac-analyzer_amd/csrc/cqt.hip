// cqt.hip — 20 s-chunk CQT chroma (K9 tuning, K10 multirate CQT, K11 chroma +
// cyclic cross-correlation lag).
//
// Replaces pitch._mean_chroma (pitch.py:55-64) =
//   librosa.feature.chroma_cqt(y, sr, bins_per_octave=36, hop_length=512).mean(axis=1)
// and pitch._cyclic_xcorr_peak (pitch.py:67-85).  CPU restatement:
// oracle/ncref.py (estimate_tuning/piptrack/pitch_tuning, cqt_mag, chroma_cqt)
// and oracle/refglue.py (cyclic_xcorr_peak).
//
// Pipeline per chunk (one launch each, all chunks of the batch at once):
//   1. decimate3_kernel x2    y_{i+1} = sqrt(2) * halfband(y_i)[::2], three levels per launch
//   2. tuning_peaks_kernel    STFT 2048/512 (Hann) -> piptrack peaks, appended per chunk
//   3. tuning_select_kernel   median(mag) -> residual histogram (0.01 bins) -> tuning index
//   4. cqt_mfma_low_kernel    octaves 0-2, cqt_mfma_kernel octaves 3-6: per octave the GEMM
//                             [frames x 1024] . [1024 x 72] on the f16 matrix cores (hi/lo split
//                             operands) -> |C|/sqrt(len) -> per-octave chroma partial rows;
//                             cqt_tail_kernel: 12-bin chroma -> inf-norm -> per-tile f64 sums
//   5. chroma_finalize_kernel mean over frames -> f32[12] per chunk
//   6. chroma_lag_kernel      argmax_k dot(src, roll(nc, -k)), wrapped to [-5, 6]
#include <algorithm>

#include "nc_block.h"
#include "nc_decim.h"
#include "nc_engine.h"
#include "nc_piptrack.h"

namespace nc {


// ------------------------------------------------------------------------------ plan
// per chunk: octave i signal at oct_off[c*7+i] (i=0 -> the chunk itself inside sig, flagged by
// a negative offset convention: we store octave 0 as a pointer offset into sig), length oct_len.
struct ChromaPlan {
  const float* sig;
  const int64_t* chunk_off;
  const int64_t* chunk_len;
  int n_chunks;
  int64_t* oct_off;   // [n][7] into ws_oct (octave 0 unused)
  int64_t* oct_len;   // [n][7]
  int* n_frames;      // [n] CQT frames (min over octaves)
  int* n_tframes;     // [n] tuning STFT frames
  int64_t* tf_base;   // [n+1] prefix of tuning frames
};

// octave lengths L_{i+1} = ceil(L_i / 2); octave buffers 64-float aligned, laid out chunk-major
__device__ __forceinline__ int64_t chunk_oct_floats(int64_t L) {
  int64_t acc = 0;
  for (int i = 1; i < 7; ++i) {
    L = (L + 1) / 2;
    acc += (L + 63) & ~63LL;
  }
  return acc;
}

// one workgroup: per-chunk octave layout and frame counts, two parallel prefix tables
// (oct_base = octave-buffer base of each chunk, tf_base = tuning-frame base)
__global__ __launch_bounds__(256) void chroma_plan_kernel(const int64_t* chunk_len, int n, int64_t* oct_off,
                                                           int64_t* oct_len, int* n_frames, int* n_tframes,
                                                           int64_t* tf_base, int64_t* oct_base,
                                                           const int* tf_skip, int64_t* tp_base) {
  block_prefix_table<256>(n, oct_base, [&](int c) { return chunk_oct_floats(chunk_len[c]); });
  block_prefix_table<256>(n, tf_base, [&](int c) { return 1 + chunk_len[c] / 512; });
  // tuning frames the tuning kernel itself computes (all but the skipped leading ones)
  block_prefix_table<256>(n, tp_base, [&](int c) { return 1 + chunk_len[c] / 512 - (tf_skip ? tf_skip[c] : 0); });
  __syncthreads();
  for (int c = threadIdx.x; c < n; c += 256) {
    int64_t L = chunk_len[c], acc = oct_base[c];
    int hop = 512, tmin = 0x7fffffff;
    for (int i = 0; i < 7; ++i) {
      oct_len[c * 7 + i] = L;
      if (i == 0) {
        oct_off[c * 7 + i] = -1;
      } else {
        oct_off[c * 7 + i] = acc;
        acc += (L + 63) & ~63LL;
      }
      tmin = min(tmin, (int)(1 + L / hop));
      hop >>= 1;
      L = (L + 1) / 2;
    }
    n_frames[c] = tmin;
    n_tframes[c] = (int)(1 + chunk_len[c] / 512);
  }
}

// ------------------------------------------------------------------------------ 1. decimation
// y_{i+1} = sqrt(2) * halfband(y_i)[::2] per chunk and level, f32 accumulation.
// Three octave levels per launch (base 0: levels 1-3 from the chunk, base 3: levels 4-6
// from level 3): a workgroup owns D3_T outputs of level base + 3 and computes the level
// base + 1 and base + 2 spans they depend on (plus the 2K halo, recomputed by both
// neighbours) in LDS, so the two inner levels are written once and never read back from
// HBM.  The arithmetic is halfband_tile<true, float>'s (nc_decim.h) bit for bit: ascending
// taps, one f32 FMA each, x sqrt(2) through f64, zeros outside each level's length.  Every
// level is staged as its even and odd phases with origin qa - 12 (qa = first output the
// next level computes), so a thread's four consecutive outputs read their 27 odd-phase
// values as 7 aligned float4 LDS loads and the centre values as one.  Measured: 1.19 ->
// 0.77 ms per bench step (isolated); in round 2, 512-output tiles (26 KB LDS) were as fast
// alone but co-resided worse with stft_mel on the other stream (step 14.5 -> 15.5 ms; 256
// (14 KB) gave 14.1 ms) -- see D3_TILE for round 4.
// Round 4, with stft_mel's LDS reserve keeping this kernel off the STFT's CUs: 128 / 256 / 512 /
// 768 / 1024 outputs per workgroup (256 threads) ran 1.40 / 0.98 / 0.82 / 0.94 / 1.01 ms per step
// isolated (six, four and three workgroups per CU past 512 by LDS), the pipelined step the same
// within its spread (profiles/r4_decimate_tile_ab.txt).  Round 5: 476 outputs, so the level-1
// pass is exactly two rounds of the 256 threads (4 T + 144 = 2048 values, 512 quads; at 512 it
// was 548 quads, a third round for 36 threads) and level 2 one (250 quads): 215.0 -> 201.2 us
// per 224 chunks, bit-identical (profiles/r5_decimate_476.txt).  Launched twice in the pipelined
// step (NC_PROBE_TWICE), decimate3 adds 0.6-0.75 ms per step: it is on the step's critical path
#ifndef D3_TILE
#define D3_TILE 476
#endif
#ifndef D3_NT
#define D3_NT 256  // threads per decimate3 workgroup
#endif
constexpr int D3_T = D3_TILE;           // level-(base + 3) outputs per decimate3 workgroup
static_assert(D3_T % 4 == 0 && D3_T >= 256, "quads per level; xmax slots are spaced 256 apart");
constexpr int D3_N1 = 4 * D3_T + 144;  // level base+1 values computed (from 4 m0 - 72)
constexpr int D3_N2 = 2 * D3_T + 48;   // level base+2 values computed (from 2 m0 - 24)
constexpr int D3_P0 = 4 * D3_T + 168;  // level base pairs staged (values from 8 m0 - 168)

// Outputs q = qa + 4i .. qa + 4i + 3 of one level from phases E/O with origin qa - 12.
__device__ __forceinline__ void d3_quad(const float* __restrict__ E, const float* __restrict__ O, int i,
                                        const float (&h)[2 * kHalfbandK + 1], float r[4]) {
  constexpr int K = kHalfbandK;
  float xo[28], xe[4];
#pragma unroll
  for (int v = 0; v < 7; ++v) {
    const float4 t = *reinterpret_cast<const float4*>(O + 4 * i + 4 * v);
    xo[4 * v] = t.x;
    xo[4 * v + 1] = t.y;
    xo[4 * v + 2] = t.z;
    xo[4 * v + 3] = t.w;
  }
  {
    const float4 t = *reinterpret_cast<const float4*>(E + 4 * i + 12);
    xe[0] = t.x;
    xe[1] = t.y;
    xe[2] = t.z;
    xe[3] = t.w;
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j <= 2 * K; ++j) {
    const int n = j - K;
    if (n != 0 && !(n & 1)) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = fmaf(h[j], n == 0 ? xe[q] : xo[q + 12 - (n + 1) / 2], acc[q]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = (float)((double)acc[q] * 1.4142135623730951);
}

// Computes level values q in [qa, qa + cnt) into the next level's phases (origin qa/2 - 12
// in pair units relative to qa: value q lands at pair (q - qa) / 2, even -> E2, odd -> O2),
// zeros outside [0, L); stores the owned span [qa + own0, qa + own0 + own_n) to dst.
__device__ __forceinline__ void d3_level(const float* E, const float* O, int cnt, int64_t qa, int64_t L,
                                         const float (&h)[2 * kHalfbandK + 1], float* E2, float* O2, float* dst,
                                         int own0, int own_n) {
  for (int i = threadIdx.x; i < cnt / 4; i += D3_NT) {
    float r[4];
    d3_quad(E, O, i, h, r);
    const int64_t q0 = qa + 4 * i;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q0 + q < 0 || q0 + q >= L) r[q] = 0.f;
    if (E2) {
      *reinterpret_cast<float2*>(E2 + 2 * i) = make_float2(r[0], r[2]);
      *reinterpret_cast<float2*>(O2 + 2 * i) = make_float2(r[1], r[3]);
    }
    if (4 * i >= own0 && 4 * i < own0 + own_n && q0 < L) {
      if (q0 + 3 < L) {
        *reinterpret_cast<float4*>(dst + q0) = make_float4(r[0], r[1], r[2], r[3]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (q0 + q < L) dst[q0 + q] = r[q];
      }
    }
  }
}

// Level base + 1 with its phases written over the level-base phases it reads: every thread
// computes its quads into registers, the workgroup syncs, then the phases go to E/O [0, N1 / 2).
// The same values as d3_level (same quads, same arithmetic).  Round 5: without the separate
// level-1 buffers the workgroup needs 16.6 KB of LDS instead of 24.8, eight waves per SIMD
// instead of six: 201.9 -> 183.7 us per 224 chunks, bit-identical; 988-output tiles of 512
// threads in the same form 195.8 (profiles/r5_decimate_476.txt)
constexpr int D3_R1 = (D3_N1 / 4 + D3_NT - 1) / D3_NT;  // level base + 1 quads per thread
__device__ __forceinline__ void d3_level1_inplace(float* E, float* O, int64_t qa, int64_t L,
                                                  const float (&h)[2 * kHalfbandK + 1], float* dst) {
  float r[D3_R1][4];
#pragma unroll
  for (int k = 0; k < D3_R1; ++k) {
    const int i = threadIdx.x + D3_NT * k;
    if (i < D3_N1 / 4) {
      d3_quad(E, O, i, h, r[k]);
      const int64_t q0 = qa + 4 * i;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q0 + q < 0 || q0 + q >= L) r[k][q] = 0.f;
      if (4 * i >= 72 && 4 * i < 72 + 4 * D3_T && q0 < L) {
        if (q0 + 3 < L) {
          *reinterpret_cast<float4*>(dst + q0) = make_float4(r[k][0], r[k][1], r[k][2], r[k][3]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (q0 + q < L) dst[q0 + q] = r[k][q];
        }
      }
    }
  }
  __syncthreads();  // every read of the level-base phases is done
#pragma unroll
  for (int k = 0; k < D3_R1; ++k) {
    const int i = threadIdx.x + D3_NT * k;
    if (i < D3_N1 / 4) {
      *reinterpret_cast<float2*>(E + 2 * i) = make_float2(r[k][0], r[k][2]);
      *reinterpret_cast<float2*>(O + 2 * i) = make_float2(r[k][1], r[k][3]);
    }
  }
}
// level base + 2 phases: after level base + 1's, 16-byte aligned
constexpr int D3_U2 = ((D3_N1 / 2) + 3) & ~3;
static_assert(D3_U2 + D3_N2 / 2 <= D3_P0 && D3_N1 / 2 <= D3_P0, "phases fit the level-base buffers");

// The level-base input of a tile is requested as D3_LD float4 loads per thread, all issued
// before any is staged (one global latency per tile instead of one per load; 276 -> 242 us
// per 224 chunks).  Walking several tiles per workgroup with the next tile's loads in
// flight during the levels measured slower (round 2: 355 against 228 us; the tile loop moves
// the taps out of SGPRs and the kernel to 105 VGPRs, four waves per SIMD instead of eight).
constexpr int D3_LD = (D3_P0 / 2 + D3_NT - 1) / D3_NT;  // float4 input loads per thread per tile

// the f32 taps by value: kernel arguments are scalar loads, so the taps stay in SGPRs
// (v_fmac takes one SGPR operand) instead of holding ~37 VGPRs for the whole kernel
struct D3Taps {
  float h[2 * kHalfbandK + 1];
};

__global__ __launch_bounds__(D3_NT) void decimate3_kernel(const float* sig, const int64_t* chunk_off,
                                                        const int64_t* oct_off, const int64_t* oct_len,
                                                        float* ws_oct, int base, D3Taps taps, float* xmax,
                                                        unsigned long long* span) {
  const Span span_(span);
  static_assert(kHalfbandK == 23, "phase windows assume 23");
  __shared__ __attribute__((aligned(16))) float e0[D3_P0], o0[D3_P0];
  __shared__ float wmax[D3_NT / 64];
  const int c = blockIdx.y;
  const int64_t m0 = (int64_t)blockIdx.x * D3_T;
  // every descriptor read up front, unconditionally: one round trip of scalar loads instead of
  // a chain (the early exit below would otherwise order the offset loads after the length's)
  const int64_t* len = oct_len + c * 7 + base;
  const int64_t L0 = len[0], L1 = len[1], L2 = len[2], L3 = len[3];
  const int64_t coff = chunk_off[c], oin = oct_off[c * 7 + base];
  const int64_t oo1 = oct_off[c * 7 + base + 1], oo2 = oct_off[c * 7 + base + 2], oo3 = oct_off[c * 7 + base + 3];
  if (m0 >= L3) return;
  const float (&h)[2 * kHalfbandK + 1] = taps.h;
  const float* in = base == 0 ? sig + coff : ws_oct + oin;
  const bool vec = ((reinterpret_cast<uintptr_t>(in) & 15) == 0);
  float* out1 = ws_oct + oo1;
  float* out2 = ws_oct + oo2;
  float* out3 = ws_oct + oo3;
  // level base of tile m0: values [8 m0 - 168, 8 m0 - 168 + 2 D3_P0), 4 values (2 pairs) per float4
  auto load_tile = [&](int64_t m0, float4 (&pf)[D3_LD]) {
    const int64_t v0 = 8 * m0 - 168;
#pragma unroll
    for (int k = 0; k < D3_LD; ++k) {
      const int u = threadIdx.x + D3_NT * k;
      const int64_t i = v0 + 4 * u;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (u < D3_P0 / 2) {
        if (vec && i >= 0 && i + 3 < L0) {
          v = *reinterpret_cast<const float4*>(in + i);
        } else if (i >= 0 && i + 3 < L0) {  // in bounds, not 16-byte aligned: four dwords, no tests
          v = make_float4(in[i], in[i + 1], in[i + 2], in[i + 3]);
        } else {
          v.x = (i >= 0 && i < L0) ? in[i] : 0.f;
          v.y = (i + 1 >= 0 && i + 1 < L0) ? in[i + 1] : 0.f;
          v.z = (i + 2 >= 0 && i + 2 < L0) ? in[i + 2] : 0.f;
          v.w = (i + 3 >= 0 && i + 3 < L0) ? in[i + 3] : 0.f;
        }
      }
      pf[k] = v;
    }
  };
  float4 pf[D3_LD];
  load_tile(m0, pf);
  {
    float m = 0.0f;  // max |level 0| over the tile's input (the MFMA CQT's f16 scale)
#pragma unroll
    for (int k = 0; k < D3_LD; ++k) {
      const int u = threadIdx.x + D3_NT * k;
      if (u < D3_P0 / 2) {
        *reinterpret_cast<float2*>(e0 + 2 * u) = make_float2(pf[k].x, pf[k].z);
        *reinterpret_cast<float2*>(o0 + 2 * u) = make_float2(pf[k].y, pf[k].w);
      }
      if (base == 0) m = fmaxf(m, fmaxf(fmaxf(fabsf(pf[k].x), fabsf(pf[k].y)), fmaxf(fabsf(pf[k].z), fabsf(pf[k].w))));
    }
    if (base == 0 && xmax) {
      m = wave_max(m);
      if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    }
    __syncthreads();
    // one maximum per workgroup, no atomics: slot c + oct_off[c][3] / 256 + blockIdx.x (distinct
    // per chunk; read back by cqt_mfma_kernel)
    if (base == 0 && xmax && threadIdx.x == 0)
    {
      float m = wmax[0];
#pragma unroll
      for (int w = 1; w < D3_NT / 64; ++w) m = fmaxf(m, wmax[w]);
      xmax[c + (base == 0 ? oo3 : oct_off[c * 7 + 3]) / 256 + blockIdx.x] = m;
    }
    // level base+1: [4 m0 - 72, +D3_N1), owned [4 m0, 4 m0 + 4 T); phases over e0/o0 [0, N1 / 2)
    d3_level1_inplace(e0, o0, 4 * m0 - 72, L1, h, out1);
    __syncthreads();
    // level base+2: [2 m0 - 24, +D3_N2), owned [2 m0, 2 m0 + 2 T); phases -> e0/o0 [U2, U2 + N2 / 2)
    d3_level(e0, o0, D3_N2, 2 * m0 - 24, L2, h, e0 + D3_U2, o0 + D3_U2, out2, 24, 2 * D3_T);
    __syncthreads();
    // level base+3: [m0, m0 + T), all owned
    d3_level(e0 + D3_U2, o0 + D3_U2, D3_T, m0, L3, h, nullptr, nullptr, out3, 0, D3_T);
  }
}

// ------------------------------------------------------------------------------ 2. tuning peaks
// piptrack(y=chunk, sr, n_fft 2048, hop 512, fmin 150, fmax 4000, threshold 0.1) inside
// estimate_tuning.  Persistent workgroups of TP_WAVES waves walk contiguous tuning frames
// (one frame per wave, the stft_mel structure: LDS twiddles, laundered lane id).  The
// peaks of a frame are appended to its chunk's region (peak_*[tf_base[c] * kPeakSlots ..])
// at an atomically reserved position: the median and the histogram that consume them
// do not depend on the order, so the result stays deterministic.
constexpr int TP_WAVES = 16;  // 14 -> 16 waves: 537 -> 495 us per 224 chunks (with the LDS Hann window)
#ifndef TP_DYN_
#define TP_DYN_ 1  // the workgroup's frames from its LDS counter (0: the static interleave; A/B)
#endif
using TpTw = StagedTw<1024>;

struct PeakArgs {
  const float* sig;
  const int64_t* chunk_off;
  const int64_t* chunk_len;
  const int* n_tframes;
  const int64_t* tf_base;
  const int64_t* tp_base;  // [n + 1] prefix of the frames this kernel computes per chunk
  int n_chunks;
  int64_t total_tframes;  // upper bound of tp_base[n]
  const float2* tw;
  const float* hann2048;
  float* peak_pitch;      // chunk c region starts at tf_base[c] * kPeakSlots
  float* peak_mag;
  int* chunk_npk;         // [n] zeroed by the launcher (or by the caller, with tf_skip)
  const int* tf_skip;     // nullable [n]: leading tuning frames whose peaks the window stage appended
  unsigned long long* span = nullptr;  // nc_profile execution span (nc_device.h)
};

__global__ __launch_bounds__(TP_WAVES * 64) void tuning_peaks_kernel(PeakArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* sh_tw = reinterpret_cast<float2*>(smem);
  const int lane0 = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  float2* sh_hann = sh_tw + ((TpTw::size + 1) & ~1);  // [1024] window pairs (h[2n], h[2n + 1])
  float2* fftbuf = sh_hann + 1024 + wave * LdsSize<1024>::value;
  __shared__ int sh_next;  // the workgroup's frame queue (WgFrameQueue)
  if (threadIdx.x == 0) sh_next = 0;
  fill_staged_tw<1024>(sh_tw, a.tw, threadIdx.x, TP_WAVES * 64);
  for (int i = threadIdx.x; i < 1024; i += TP_WAVES * 64) sh_hann[i] = reinterpret_cast<const float2*>(a.hann2048)[i];
  __syncthreads();
  // this lane's Hann taps held across frames (the stft_mel form, round 5): no LDS reads per frame
  float2 hw[16];
  lds_read16_strided<0, 64 * 8>(hw, lds_addr(sh_hann + fft_in_lane(lane0)));
  const int64_t n_groups = (a.total_tframes + TP_WAVES - 1) / TP_WAVES;
  const int64_t gb = n_groups * blockIdx.x / gridDim.x, ge = n_groups * (blockIdx.x + 1) / gridDim.x;
  // The workgroup's work-list frames [f0, f1) go to its waves one at a time (WgFrameQueue, as in
  // stft_mel); a wave's frames gf rise: their chunk is tracked forward, its bounds and
  // descriptors reloaded only when gf crosses into a later chunk (no binary search and
  // dependent loads per frame).  TP_DYN_=0: the static interleave (wave w: frames 16 G + w)
  const int64_t f0 = gb * TP_WAVES, f1 = std::min<int64_t>(ge * TP_WAVES, a.total_tframes);
  WgFrameQueue fq(&sh_next, lane0);
  int c = -1, nt = 0, skip = 0;
  int64_t cb = 0, ce = -1, coff = 0, clen = 0, ctf = 0;
  for (int64_t grp = gb; TP_DYN_ || grp < ge; ++grp) {
    const int64_t gf = TP_DYN_ ? f0 + fq.take(lane0) : grp * TP_WAVES + wave;
    if (gf >= (TP_DYN_ ? f1 : a.total_tframes)) break;
    if (gf >= ce) {
      if (c < 0) {
        int lo = 0, hi = a.n_chunks - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (a.tp_base[mid] <= gf) lo = mid;
          else hi = mid - 1;
        }
        c = lo;
      } else {
        do ++c;
        while (c + 1 < a.n_chunks && a.tp_base[c + 1] <= gf);
      }
      c = uniform32(c);
      cb = uniform64(a.tp_base[c]);
      ce = uniform64(c + 1 < a.n_chunks ? a.tp_base[c + 1] : INT64_MAX);
      // frames [0, tf_skip[c]) of the chunk were done by the window stage: the work list is
      // the remaining frames only, so the persistent workgroups stay balanced
      skip = uniform32(a.tf_skip ? a.tf_skip[c] : 0);
      nt = uniform32(a.n_tframes[c]);
      coff = uniform64(a.chunk_off[c]);
      clen = uniform64(a.chunk_len[c]);
      ctf = uniform64(a.tf_base[c]);
    }
    const int t = (int)(gf - cb) + skip;
    if (t >= nt) continue;
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int jin = fft_in_lane(lane);  // this lane's stage-1 butterfly: samples x[2 (jin + 64 r)]
    const int64_t off = coff;
    const float* x = a.sig + off;
    const int64_t L = clen;
    const int64_t s0 = (int64_t)t * 512 - 1024;
    FftIn<1024> in;
    if (s0 >= 0 && s0 + 2048 <= L) {
      float2 xv[16];
      if ((off & 1) == 0) {
        const float2* x2 = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
        for (int r = 0; r < 16; ++r) xv[r] = x2[jin + 64 * r];
      } else {
        // a chunk at an odd sample: two dword loads per pair, no bounds tests (stft_mel)
        const float* xs = x + s0;
#pragma unroll
        for (int r = 0; r < 16; ++r) xv[r] = make_float2(xs[2 * (jin + 64 * r)], xs[2 * (jin + 64 * r) + 1]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) in[0][r] = make_float2(xv[r].x * hw[r].x, xv[r].y * hw[r].y);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = jin + 64 * r;
        const int64_t i0 = s0 + 2 * n;
        const float x0 = (i0 >= 0 && i0 < L) ? x[i0] : 0.0f;
        const float x1 = (i0 + 1 >= 0 && i0 + 1 < L) ? x[i0 + 1] : 0.0f;
        in[0][r] = make_float2(x0 * a.hann2048[2 * n], x1 * a.hann2048[2 * n + 1]);
      }
    }
    // stages 1-2 through LDS, the last stage on mirror-paired butterflies, then the real split
    // and |X| straight from registers (stft_mel structure)
    stockham_stage_regs<1024, 16, 1, 64, false, 0, 0>(in, fftbuf, sh_tw, jin);
    stockham_stage<1024, 16, 16, 64, false, 0, 0>(fftbuf, sh_tw, lane);
    float2 v[4][4];
    fft1024_last_mirror<TpTw::s3>(fftbuf, sh_tw, lane, v);
    // |2X|^2 (the split without its 0.5 scalings: piptrack's decisions are scale-free, and its
    // magnitudes come out as exactly 2|X|, as in stft_mel's shared frames) into LDS only where
    // the peak stencil reads it (bins kPipLo-1 .. kPipHi+1); the frame max is sqrt(max |2X|^2)
    // (the correctly rounded sqrt is monotonic), so the other 2/3 of the bins need no square root
    float* S = reinterpret_cast<float*>(fftbuf);  // (all Z reads precede)
    float pmax = 0.0f;
    rsplit_mirror<TpTw::split, false>(v, sh_tw, lane, [&](int k, float2 X, float2 XN) {
      const float p1 = fmaf(X.x, X.x, X.y * X.y), p2 = fmaf(XN.x, XN.x, XN.y * XN.y);
      // k <= 512 covers the stencil's bins (<= kPipHi + 1) and 1024 - k >= 512 never does:
      // the low half is stored unconditionally (no exec-masked branch per pair)
      S[k] = p1;
      pmax = fmaxf(pmax, fmaxf(p1, p2));
    });
    const float mx = __fsqrt_rn(wave_max_u(pmax));
    // |X| over the stencil's bins, in place (6 per lane)
#pragma unroll
    for (int q = 0; q < (kPipHi - kPipLo + 3 + 63) / 64; ++q) {
      const int k = kPipLo - 1 + 64 * q + lane;
      if (64 * (q + 1) <= kPipHi - kPipLo + 3 || k <= kPipHi + 1) S[k] = __fsqrt_rn(S[k]);  // test the last round only
    }
    piptrack_append([&](int k) { return S[k]; }, mx, lane, &a.chunk_npk[c], a.peak_pitch + ctf * kPeakSlots,
                    a.peak_mag + ctf * kPeakSlots, reinterpret_cast<int*>(S + kPipKpk));
  }
}

// ------------------------------------------------------------------------------ 3. tuning select
// 1024 threads per chunk: 79.8 -> 34.9 us per 224 chunks against 256 (the passes are
// latency-bound loops over the peak list; wave-aggregated top-byte counts, which remove
// the LDS same-address conflicts, measured no better)
constexpr int TS_NT = 1024;
__device__ __forceinline__ int tuning_bin(float r) {
  // np.histogram(residual, linspace(-0.5, 0.5, 101)) bin of r (exact edge comparisons in f64)
  const double rd = (double)r;
  int j = (int)floor((rd + 0.5) * 100.0);
  j = max(0, min(99, j));
  auto edge = [](int i) { return i == 100 ? 0.5 : (double)i * (1.0 / 100.0) + (-0.5); };
  while (j > 0 && rd < edge(j)) --j;
  while (j < 99 && rd >= edge(j + 1)) ++j;
  return j;
}

__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u >> 31) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funkey(unsigned k) {
  return __uint_as_float((k >> 31) ? (k & 0x7fffffffu) : ~k);
}

__device__ __forceinline__ int wave_incl_scan_i(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// One workgroup per chunk: median of the peak magnitudes (4-pass 8-bit radix select over
// the chunk's compact peak list, plus one pass for the upper middle of an even count),
// then the 100-bin residual histogram and its first argmax (librosa estimate_tuning /
// pitch_tuning, oracle/ncref.py).
// The CQT kernels' per-(chunk, octave) f16 split exponent: 2^ex scales the octave's samples so
// their largest (bounded by the chunk's max |level 0| times the octave's gain) sits below 2^13
struct OctScale {
  const float* xmax;      // decimate3 workgroup maxima of |level 0| (slot c + oct_off[c][3] / 256 + tile)
  const int64_t* oct_off;
  const int64_t* oct_len;
  int d3_span;            // level-3 outputs per decimate3 workgroup
  float gpow[7];
  int* oct_ex;            // [n][7]
};

template <int NT>
__global__ __launch_bounds__(NT) void tuning_select_kernel(const float* peak_pitch, const float* peak_mag,
                                                           const int* chunk_npk, const int64_t* tf_base,
                                                           int* tuning_idx, float* tuning_val, int* tuning_margin,
                                                           OctScale os, unsigned long long* span) {
  const Span span_(span);
  if (threadIdx.x < 64) {  // wave 0: the chunk's octave exponents (the CQT kernels read them)
    const int c = blockIdx.x, lane = threadIdx.x;
    const int64_t l3 = os.oct_len[c * 7 + 3];
    const int ntl = (int)((l3 + os.d3_span - 1) / os.d3_span);
    const float* xm = os.xmax + c + os.oct_off[c * 7 + 3] / 256;
    float m0 = 0.0f;
    for (int i = lane; i < ntl; i += 64) m0 = fmaxf(m0, xm[i]);
    const float m = wave_max_u(m0);
    if (lane < 7) {
      const float mx = m * os.gpow[lane];
      int ex = 0;
      if (mx > 0.0f) {
        int e;
        frexpf(mx, &e);  // mx < 2^e
        ex = min(13 - e, 100);
      }
      os.oct_ex[c * 7 + lane] = ex;
    }
  }
  __shared__ BlockScratch<NT> bs;
  __shared__ int hist[256];
  __shared__ int counts[100];
  __shared__ int sel[2];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t base = tf_base[c] * kPeakSlots;
  const float* mg = peak_mag + base;
  const float* pt = peak_pitch + base;
  const int N = chunk_npk[c];
  float thr = 0.0f;
  if (N > 0) {
    int kk = (N - 1) / 2;
    unsigned prefix = 0, mask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = tid; i < 256; i += NT) hist[i] = 0;
      __syncthreads();
      for (int i = tid; i < N; i += NT) {
        const unsigned key = fkey(mg[i]);
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
      }
      __syncthreads();
      if (wave == 0) {
        const int h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
        const int s = h0 + h1 + h2 + h3;
        const int incl = wave_incl_scan_i(s), excl = incl - s;
        if (excl <= kk && kk < incl) {
          int r = kk - excl, d = 4 * lane;
          const int hh[4] = {h0, h1, h2, h3};
          for (int q = 0; q < 4; ++q) {
            if (r < hh[q]) {
              d = 4 * lane + q;
              break;
            }
            r -= hh[q];
          }
          sel[0] = d;
          sel[1] = r;
        }
      }
      __syncthreads();
      prefix |= (unsigned)sel[0] << shift;
      mask |= 255u << shift;
      kk = sel[1];
      __syncthreads();
    }
    const float lo = funkey(prefix);
    if (N & 1) {
      thr = lo;
    } else {
      // upper middle: lo again if at least (N/2 + 1) keys are <= lo, else the smallest key above it
      int le = 0;
      float above = INFINITY;
      for (int i = tid; i < N; i += NT) {
        const float v = mg[i];
        if (fkey(v) <= prefix) ++le;
        else above = fminf(above, v);
      }
      le = block_sum_i<NT>(le, bs);
      above = (float)(-block_max(-(double)above, bs));
      const float hi = (le >= N / 2 + 1) ? lo : above;
      thr = (lo + hi) / 2.0f;
    }
  }
  for (int i = tid; i < 100; i += NT) counts[i] = 0;
  __syncthreads();
  int nsel = 0;
  for (int i = tid; i < N; i += NT) {
    const float m = mg[i], p = pt[i];
    if (m >= thr && p > 0.0f) {
      const float o = log2f(p / 27.5f);
      float r = fmodf(36.0f * o, 1.0f);
      if (r < 0.0f) r += 1.0f;
      if (r >= 0.5f) r -= 1.0f;
      atomicAdd(&counts[tuning_bin(r)], 1);
      ++nsel;
    }
  }
  nsel = block_sum_i<NT>(nsel, bs);
  if (tid == 0) {
    int best = 50;
    if (nsel > 0) {
      best = 0;
      for (int j = 1; j < 100; ++j)
        if (counts[j] > counts[best]) best = j;
    }
    tuning_idx[c] = best;
    tuning_val[c] = (float)((double)best * (1.0 / 100.0) + (-0.5));
    if (tuning_margin) {  // decision margin: argmax count minus the runner-up's (0 = tie, first index won)
      int second = -1;
      for (int j = 0; j < 100; ++j)
        if (j != best) second = max(second, counts[j]);
      tuning_margin[c] = nsel > 0 ? counts[best] - second : 0;
    }
  }
}

// ------------------------------------------------------------------------------ 4. CQT on MFMA
// The CQT response is linear in the frame: C_j[t] = sum_b fb[j][b] rfft(x_t)[b] =
// sum_n x_t[n] h_j[n] with h_j[n] = sum_b fb[j][b] e^{-2 pi i b n / 1024} (nc_tables.cpp).
// Per octave that is a real GEMM [frames x 1024] . [1024 x 72] (Re and Im of the 36 rows),
// run on the f16 matrix cores with both operands split into hi + lo halves (x = xh + xl,
// products xh.hh + xh.hl + xl.hh, f32 accumulation): 22 significant bits per operand, so
// |C| matches an f32 FFT to ~1e-6 of the frame's largest bin.  The frame operand is scaled
// by 2^ex with max|y_o| * 2^ex < 2^13 (max|y_0| from decimate3, bounded per octave by
// (sqrt(2) sum|h|)^o) and the filters by 2^e_j; C = acc * 2^-(ex + e_j) exactly.
//
// Octaves 3-6 (hop <= 64, cqt_mfma_kernel): one workgroup per (chunk, 32-frame tile), one
// wave per octave: 2 row tiles x 5 column tiles x 3 products = 30 MFMA 16x16x32 per k-step
// of 32 taps, 32 k-steps.  The tile's span (31 hop + 1024 samples) is split once into an LDS
// image that every k-step's fragments read; the filter slices (one k-step: 10 fragments x
// 1 KB) stream through a two-slot LDS ring by LDS-DMA, with one raw s_barrier per k-step.
// 52 KB of LDS: three workgroups per CU, whose k-steps interleave freely (64-frame tiles with
// padded images until round 5: 78 KB, two per CU).  Octaves 0-2 (hop
// >= 128, cqt_mfma_low_kernel below): their spans do not fit LDS as images.  Both write
// per-(frame, octave) chroma partial rows; cqt_tail_kernel finishes the frames.
//
// Measured and not kept (round 2, per 224 chunks): two tiles per workgroup
// sharing a 2 / 3 / 4-slot ring 809 / 822 / 812-822 against 753-770 us; two or four k-steps
// per barrier 780-869 against 722-727 us; the next k-step's A fragments read under this
// step's MFMAs 748-765 against 730-745 us; octave 2 in a workgroup of its own 888-1012
// against 879 us; the FFT CQT kernel for octaves 0-2 866 against 816-856 us (removed in
// round 3).
constexpr int CM_FR = 64;                          // frames per cqt_tail / partial-sum tile
constexpr int CM_RT = CM_FR / 16;                  // row tiles per wave
// Round 5: 32-frame tiles with swizzled (unpadded) images need 52 KB of LDS, three workgroups
// (twelve waves) per CU instead of two at 78 KB: 343.0 -> 326.5 us per 224 chunks, bit-identical;
// 32 frames with the pads (two per CU) 381.2, 64 frames swizzled 348.5, 64 unpadded (bank
// conflicts) 345.3 (profiles/r5_cqt_high_tiles.txt)
#ifndef CH_FR_
#define CH_FR_ 32
#endif
#ifndef CH_MINB_
#define CH_MINB_ 3
#endif
constexpr int CH_FR = CH_FR_;                      // frames per cqt_mfma_kernel workgroup tile
constexpr int CH_RT = CH_FR / 16;                  // its row tiles per wave
static_assert(CH_RT == 2 || CH_RT == 4, "tile rows");
constexpr int CM_KS = kCqtNfft / 32;               // k-steps of 32 taps
constexpr int CM_NT = 5;                           // column tiles (72 of 80 columns used)
constexpr int CM_R = 2;                            // filter-slice ring slots
constexpr int CM_SLICE = CM_NT * 2 * 64;           // uint4 fragments per k-step slice
constexpr int CM_LO = 3;                           // first octave of cqt_mfma_kernel
constexpr int CM_NW = 7 - CM_LO;                   // waves (octaves) per workgroup
constexpr int CM_NTH = CM_NW * 64;
constexpr int CM_GQ = (CM_NT * 2 + CM_NW - 1) / CM_NW;  // filter DMA pieces per wave per slice
typedef _Float16 cm_half8 __attribute__((ext_vector_type(8)));
typedef float cm_f4 __attribute__((ext_vector_type(4)));
typedef unsigned cm_u4 __attribute__((ext_vector_type(4)));

// s_waitcnt immediate for vmcnt(n) alone (vmcnt [3:0] + [15:14]; expcnt, lgkmcnt at maximum)
__host__ __device__ constexpr int cm_vmcnt(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70 | 0xf00; }

// LDS images: span 63 hop + 1024 samples as f16 hi then lo, with 16 halves of padding after
// every hop samples when hop >= 32 (row r starts at r (hop + pad)); a row's 8-sample piece
// never straddles a pad.  ds_read_b128 serves a wave in the lane groups {0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31}, ... (MI355X_MICROARCH.md, LDS table): a group holds 8 rows at one k
// offset and 8 rows at the next, and with these pads its 16 pieces fall on distinct banks for
// every octave and k-step (the round-2 pads, 8 halves when hop >= 16, gave 2-way conflicts
// for octaves 3-5)
__host__ __device__ constexpr int cm_hop(int o) { return 512 >> o; }
#ifndef CH_PAD_
#define CH_PAD_ 16
#endif
// CH_SWZ_: no pads; instead 16-byte piece P of a hop-64 / hop-32 image sits at P ^ cm_swz(P),
// an XOR of its low four bits keyed by its 256-byte block (conflict-free for every fragment
// read by the bank model above, tests/test_lds_layout_cpu.py); hop 16 and 8 are conflict-free
// unpadded
#ifndef CH_SWZ_
#define CH_SWZ_ 1
#endif
__host__ __device__ constexpr int cm_pad(int o) { return cm_hop(o) >= 32 && !CH_SWZ_ ? CH_PAD_ : 0; }
// (key table, block-index mask) of octave o's swizzle: h[(P >> 4) & m] = (K >> 4 ((P >> 4) & m)) & 15
__host__ __device__ constexpr unsigned cm_swz_k(int o) { return !CH_SWZ_ ? 0u : cm_hop(o) == 64 ? 0xC638u : cm_hop(o) == 32 ? 0xF8u : 0u; }
__host__ __device__ constexpr int cm_swz_m(int o) { return cm_hop(o) == 64 ? 3 : 1; }
__host__ __device__ __forceinline__ int cm_phys(int P, unsigned K, int m) { return P ^ (int)((K >> (((P >> 4) & m) << 2)) & 15u); }
__host__ __device__ constexpr int cm_span(int o) { return (CH_FR - 1) * cm_hop(o) + kCqtNfft; }
__host__ __device__ constexpr int cm_img(int o) {  // halves per hi (or lo) image, 16-byte multiple
  // (whole 256-byte blocks when swizzled: a piece of the last block may move anywhere in it)
  return cm_swz_k(o) ? (cm_span(o) + 127) & ~127 : (cm_span(o) + (cm_span(o) / cm_hop(o)) * cm_pad(o) + 7) & ~7;
}
__host__ __device__ constexpr int cm_aoff(int o) {  // byte offset of octave o's image pair
  return o <= CM_LO ? 0 : cm_aoff(o - 1) + 4 * cm_img(o - 1);
}
// K-loop LDS: filter ring [CM_R][CM_SLICE] uint4 | images.  Epilogue overlay: octave rows
// [CM_NW][CH_FR][36] f32
constexpr int CM_BBYTES = CM_R * CM_SLICE * 16;
// Image pieces per lane whose loads are issued together.  One session, cqt_chroma per 224
// chunks: 1 / 2 / 4 / 8 -> 751-753 / 739 / 744-745 / 743 us.
constexpr int CM_IMGU = 4;
constexpr int CM_KBYTES = CM_BBYTES + cm_aoff(7);
constexpr int CM_MBYTES = CM_NW * CH_FR * kCqtFilt * 4;
size_t cqm_lds_bytes() { return CM_KBYTES > CM_MBYTES ? CM_KBYTES : CM_MBYTES; }

struct CqmArgs {
  const float* sig;
  const int64_t* chunk_off;
  const int64_t* oct_off;
  const int64_t* oct_len;
  const int* n_frames;
  const int* tuning_idx;
  const float* ws_oct;
  const int64_t* tf_base;
  const uint4* bfrag;    // Tables::cqm_b
  const int* bexp;       // Tables::cqm_bexp
  const float* cqt_isl;
  const int* oct_ex;     // [n][7] f16 split exponents (tuning_select_kernel, OctScale)
  float* gpart;          // [tf_base[c] + t][7][12] octave chroma partial rows
  unsigned long long* span = nullptr;
};

// One LDS-DMA instruction: 16 bytes per lane from gsrc to lds_dst + 16 lane (lds_dst
// wave-uniform).  Inline asm rather than __builtin_amdgcn_global_load_lds: the compiler
// drains vmcnt(0) before any later LDS read when it sees the builtin; the kernel counts its
// own vmcnt instead.
__device__ __forceinline__ void cm_dma16(const void* gsrc, const void* lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr(lds_dst)))
               : "memory");
}

// Fragment reads issued by asm with no wait, retired by counted waits (cm_wait) that also tie
// the fragments' registers, so no MFMA can read one early.  The compiler's scheduler sinks
// each column tile's compiler-issued B reads next to that tile's MFMAs, with an
// s_waitcnt lgkmcnt between every two tiles: one exposed LDS latency per column tile.
// Only these reads are outstanding on lgkmcnt inside the k-loop (the loop top drains it).
template <int OFF>
__device__ __forceinline__ void cm_rd(cm_u4& d, uint32_t a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(d) : "v"(a), "i"(OFF) : "memory");
}
template <int N>
__device__ __forceinline__ void cm_wait(cm_u4& x, cm_u4& y) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(x), "+v"(y) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void cm_wait(cm_u4& x, cm_u4& y, cm_u4& z, cm_u4& w) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "i"(N) : "memory");
}

// 8 samples -> f16 hi (f32 truncated to 11 significant bits: exact in f16) and lo (the
// exact f32 remainder, rounded toward zero)
__device__ __forceinline__ void cm_split(const float (&v)[8], float s, cm_half8& hi, cm_half8& lo) {
  cm_u4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x0 = v[2 * j] * s, x1 = v[2 * j + 1] * s;
    const float h0 = __uint_as_float(__float_as_uint(x0) & 0xffffe000u);
    const float h1 = __uint_as_float(__float_as_uint(x1) & 0xffffe000u);
    h[j] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(h0, h1));
    l[j] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(x0 - h0, x1 - h1));
  }
  hi = __builtin_bit_cast(cm_half8, h);
  lo = __builtin_bit_cast(cm_half8, l);
}

__global__ __launch_bounds__(CM_NTH, CH_MINB_) void cqt_mfma_kernel(CqmArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* sB = reinterpret_cast<uint4*>(smem);  // [CM_R][CM_SLICE]
  // logical (tile, chunk), tile fastest, XCD-contiguous: a chunk's tiles share one L2 (and its
  // tuning's filter slices): FETCH_SIZE 76.6 -> 53.8 MiB per 112 chunks, time unchanged
  const unsigned lg = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int bx = (int)(lg % gridDim.x);
  const int c = (int)(lg / gridDim.x);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int oct = CM_LO + wave;
  // every descriptor read up front, unconditionally: one round trip of scalar loads
  const int T = a.n_frames[c], ti = a.tuning_idx[c], ex = a.oct_ex[c * 7 + oct];
  const int64_t yoff = a.oct_off[c * 7 + oct], Ly = a.oct_len[c * 7 + oct];
  const int t0 = bx * CH_FR;
  if (t0 >= T) return;
  const int nfr = min(CH_FR, T - t0);
  const uint4* bsrc = a.bfrag + (size_t)ti * (CM_KS * CM_SLICE);
  // the first filter slice is in flight while the image is built
  auto fetch_slice = [&](int ks) {
#pragma unroll
    for (int q = 0; q < CM_GQ; ++q) {
      int i = wave + CM_NW * q;
      if (i >= CM_NT * 2) i = wave;  // duplicate of this wave's first piece (same bytes, same place)
      cm_dma16(bsrc + ks * CM_SLICE + i * 64 + lane, sB + (ks % CM_R) * CM_SLICE + i * 64);
    }
  };
  fetch_slice(0);

  // this wave's octave: rows t0 .. t0 + 63, row t at sample t hop - 512
  const float* y = a.ws_oct + yoff;
  const int hop = 512 >> oct;
  const float sx = ldexpf(1.0f, ex);
  const int64_t s0 = (int64_t)t0 * hop - 512;  // first sample of the tile's span
  const int S = (CH_FR - 1) * hop + kCqtNfft;
  const bool vec = s0 >= 0 && s0 + S <= Ly && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
  const int kq = 8 * (lane >> 4);

  // the span, split once (rows past T - 1 read real or zero samples and are discarded)
  constexpr int aoffs[8] = {cm_aoff(0), cm_aoff(1), cm_aoff(2), cm_aoff(3), cm_aoff(4), cm_aoff(5), cm_aoff(6), cm_aoff(7)};
  const int pad = cm_pad(oct);
  const int img = cm_img(oct);
  constexpr unsigned swk[8] = {cm_swz_k(0), cm_swz_k(1), cm_swz_k(2), cm_swz_k(3), cm_swz_k(4), cm_swz_k(5), cm_swz_k(6), cm_swz_k(7)};
  const unsigned sk = swk[oct];
  const int sm = cm_swz_m(oct);
  _Float16* aimg = reinterpret_cast<_Float16*>(smem + CM_BBYTES + aoffs[oct]);
  int ib = lane;
  if (vec) {
    // CM_IMGU pieces per lane loaded before any is split: one load latency per batch instead
    // of one per piece (the accumulators are not live yet, so the registers are free)
    for (; ib + (CM_IMGU - 1) * 64 < S / 8; ib += CM_IMGU * 64) {
      float4 u[CM_IMGU][2];
#pragma unroll
      for (int k = 0; k < CM_IMGU; ++k) {
        const float4* p = reinterpret_cast<const float4*>(y + s0 + 8 * (ib + k * 64));
        u[k][0] = p[0];
        u[k][1] = p[1];
      }
#pragma unroll
      for (int k = 0; k < CM_IMGU; ++k) {
        const int i = ib + k * 64;
        const float v[8] = {u[k][0].x, u[k][0].y, u[k][0].z, u[k][0].w, u[k][1].x, u[k][1].y, u[k][1].z, u[k][1].w};
        cm_half8 h, l;
        cm_split(v, sx, h, l);
        const int pos = CH_SWZ_ ? 8 * cm_phys(i, sk, sm) : 8 * i + (8 * i / hop) * pad;
        *reinterpret_cast<cm_half8*>(aimg + pos) = h;
        *reinterpret_cast<cm_half8*>(aimg + img + pos) = l;
      }
    }
  }
  for (int i = ib; i < S / 8; i += 64) {
    float v[8];
    if (vec) {
      const float4 u0 = *reinterpret_cast<const float4*>(y + s0 + 8 * i);
      const float4 u1 = *reinterpret_cast<const float4*>(y + s0 + 8 * i + 4);
      v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w;
      v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t q = s0 + 8 * i + j;
        v[j] = (q >= 0 && q < Ly) ? y[q] : 0.0f;
      }
    }
    cm_half8 h, l;
    cm_split(v, sx, h, l);
    const int pos = CH_SWZ_ ? 8 * cm_phys(i, sk, sm) : 8 * i + (8 * i / hop) * pad;
    *reinterpret_cast<cm_half8*>(aimg + pos) = h;
    *reinterpret_cast<cm_half8*>(aimg + img + pos) = l;
  }
  int abase[CH_RT];
#pragma unroll
  for (int rt = 0; rt < CH_RT; ++rt)
    abase[rt] = CH_SWZ_ ? ((16 * rt + (lane & 15)) * hop + kq) / 8  // the fragment's first piece
                        : (16 * rt + (lane & 15)) * (hop + pad) + kq + (kq / hop) * pad;

  cm_f4 acc[CH_RT][CM_NT];
#pragma unroll
  for (int rt = 0; rt < CH_RT; ++rt)
#pragma unroll
    for (int nt = 0; nt < CM_NT; ++nt) acc[rt][nt] = cm_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int ks = 0; ks < CM_KS; ++ks) {
    // retire this wave's DMA of slice ks (vmcnt(0): nothing younger is in flight, and a
    // counted wait over mixed LDS-DMA raced in round 2); the barrier makes
    // every wave's pieces visible and ends every read of the slot slice ks + 1 reuses
    __builtin_amdgcn_s_waitcnt(cm_vmcnt(0));
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the image writes (first step)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ks + 1 < CM_KS) fetch_slice(ks + 1);
    // A fragments of k-step ks (this wave's own image: written by this wave only, and LDS
    // operations of one wave complete in order, so no barrier guards them), then the B
    // fragments two column tiles ahead of their MFMAs
    const int kt = 32 * ks + (32 * ks / hop) * pad;
    const uint32_t sbl = lds_addr(sB + (ks % CM_R) * CM_SLICE + lane);
    cm_u4 a4[CH_RT], l4[CH_RT], b[CM_NT][2];
    static_assert(CM_NT == 5, "fragment schedule");
#pragma unroll
    for (int rt = 0; rt < CH_RT; ++rt)
      cm_rd<0>(a4[rt], lds_addr(aimg + (CH_SWZ_ ? 8 * cm_phys(abase[rt] + 4 * ks, sk, sm) : abase[rt] + kt)));
#pragma unroll
    for (int rt = 0; rt < CH_RT; ++rt)
      cm_rd<0>(l4[rt], lds_addr(aimg + img + (CH_SWZ_ ? 8 * cm_phys(abase[rt] + 4 * ks, sk, sm) : abase[rt] + kt)));
    cm_rd<0 * 1024>(b[0][0], sbl);
    cm_rd<1 * 1024>(b[0][1], sbl);
    cm_rd<2 * 1024>(b[1][0], sbl);
    cm_rd<3 * 1024>(b[1][1], sbl);
    cm_rd<4 * 1024>(b[2][0], sbl);
    cm_rd<5 * 1024>(b[2][1], sbl);
    if constexpr (CH_RT == 4) {
      cm_wait<4>(a4[0], a4[1], a4[2], a4[3]);  // A + tile 0 landed; tiles 1, 2 in flight
      cm_wait<4>(l4[0], l4[1], l4[2], l4[3]);
    } else {
      cm_wait<4>(a4[0], a4[1], l4[0], l4[1]);
    }
    cm_half8 ah[CH_RT], al[CH_RT];
#pragma unroll
    for (int rt = 0; rt < CH_RT; ++rt) {
      ah[rt] = __builtin_bit_cast(cm_half8, a4[rt]);
      al[rt] = __builtin_bit_cast(cm_half8, l4[rt]);
    }
    auto tile = [&](int nt) {
      const cm_half8 bh = __builtin_bit_cast(cm_half8, b[nt][0]);
      const cm_half8 bl = __builtin_bit_cast(cm_half8, b[nt][1]);
#pragma unroll
      for (int rt = 0; rt < CH_RT; ++rt) {
        acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt], bh, acc[rt][nt], 0, 0, 0);
        acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt], bl, acc[rt][nt], 0, 0, 0);
        acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[rt], bh, acc[rt][nt], 0, 0, 0);
      }
    };
    cm_wait<4>(b[0][0], b[0][1]);
    tile(0);
    cm_rd<6 * 1024>(b[3][0], sbl);
    cm_rd<7 * 1024>(b[3][1], sbl);
    cm_wait<4>(b[1][0], b[1][1]);
    tile(1);
    cm_rd<8 * 1024>(b[4][0], sbl);
    cm_rd<9 * 1024>(b[4][1], sbl);
    cm_wait<4>(b[2][0], b[2][1]);
    tile(2);
    cm_wait<2>(b[3][0], b[3][1]);
    tile(3);
    cm_wait<0>(b[4][0], b[4][1]);
    tile(4);
  }
  __syncthreads();  // every wave's last ring / image reads done before the rows overlay them

  // |C| per (frame, row) into this wave's [64][36] region
  float* mg = reinterpret_cast<float*>(smem) + wave * (CH_FR * kCqtFilt);
  {
    const float oscale = (float)(1 << (oct >> 1)) * ((oct & 1) ? 0x1.6a09e6p+0f : 1.0f);
    const float* isl = a.cqt_isl + ti * kCqtBins + (kCqtBins - kCqtFilt * (oct + 1));
    const int* bx = a.bexp + ti * kCqtFilt;
    const int col = lane & 15;
    const float inv0 = ldexpf(1.0f, -(ex + bx[col])), inv1 = ldexpf(1.0f, -(ex + bx[16 + col]));
    const float inv2 = ldexpf(1.0f, -(ex + bx[32 + (col & 3)]));
    const float il0 = isl[col], il1 = isl[16 + col], il2 = isl[32 + (col & 3)];
#pragma unroll
    for (int rt = 0; rt < CH_RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int fr = 16 * rt + 4 * (lane >> 4) + i;  // row within the tile
        float* m = mg + fr * kCqtFilt;
        m[col] = hypotf(acc[rt][0][i] * inv0 * oscale, acc[rt][1][i] * inv0 * oscale) * il0;
        m[16 + col] = hypotf(acc[rt][2][i] * inv1 * oscale, acc[rt][3][i] * inv1 * oscale) * il1;
        const float im = __shfl_down(acc[rt][4][i], 4, 16);
        if (col < 4) m[32 + col] = hypotf(acc[rt][4][i] * inv2 * oscale, im * inv2 * oscale) * il2;
      }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // the wave reads back only its own rows
  __builtin_amdgcn_wave_barrier();
  // this octave's share of the 12 chroma bins: bins 3c-1, 3c, 3c+1 (mod 36), ascending
  float* gp = a.gpart + (a.tf_base[c] + t0) * (7 * 12) + (6 - oct) * 12;
  for (int q = lane; q < nfr * 12; q += 64) {
    const int fl = q / 12, cc = q - 12 * fl;
    const float* m = mg + fl * kCqtFilt;
    gp[fl * (7 * 12) + cc] = cc == 0 ? (m[0] + m[1]) + m[35] : (m[3 * cc - 1] + m[3 * cc]) + m[3 * cc + 1];
  }
}

// ---- Octaves 0-2 (hop >= 128): their 64-frame spans (9-33 K samples) do not fit LDS as images,
// but row t + 1 at k-step ks equals row t at k-step ks + G (G = hop / 32): the M = 1024 / hop
// k-steps {g + G q : q < M} of "group" g read one block of 64 + M - 1 row pieces (32 samples
// each), row r of step q being block row r + q.  The k-steps run group by group, so each sample
// is fetched once per tile.  Round 5 rebuilt the kernel around one 64-frame
// tile per wave (the round-2 kernel ran two waves of 32 rows per tile and split every A fragment
// from f32 at each of the M k-steps that read its row: 4.8 VALU per MFMA):
//  * a wave owns a whole tile (4 row tiles x 5 column tiles x 3 products = 60 MFMAs per k-step);
//    two tiles of one (chunk, octave) per workgroup share the filter slices;
//  * the block of group g + 1 is loaded into registers at group g's first step and split ONCE
//    (cm_split, the same values) into this wave's f16 hi / lo image at the group's last step, so
//    a k-step's A fragments are plain ds_read_b128s at immediate offsets;
//  * filter slices go through a two-slot LDS ring by LDS-DMA, slice n + 1 requested at step n
//    and retired by a counted vmcnt at step n + 1's top (the block loads stay in flight): every
//    wave issues the same vector-memory sequence (5 slice pieces per step, 10 block loads at a
//    group's first step), so the count of younger operations is static per position in the
//    group (C2::younger).  The counted wait relies on vmcnt retiring in issue order across
//    global_load_lds and global_load: round 6 measured that directly (tools/probe/vmcnt_order.hip:
//    an LDS-DMA piece from an HBM-cold line, then 4 L2-hot register loads, vmcnt(4), the LDS read;
//    and the reverse, a cold register load then 4 hot LDS-DMA pieces: 0 stale of 3.4e8 lane-trials
//    each, profiles/r6_vmcnt_order.txt), as MI355X_MICROARCH.md states.  (Round 5 had blamed out-of-
//    order retirement for NaNs from a counted wait on the block loads; the block wait stays
//    vmcnt(0).  C2_SAFE_=1, vmcnt(0) wherever a block load is younger than the slice, measured
//    the same: 353.3 against 352.7 us per 224 chunks, profiles/r6_var_bench.txt);
//  * block loads are dword-aligned dwordx4 (gfx950 serves unaligned global loads), so an
//    unaligned chunk issues the same instructions; an edge tile loads clamped pieces and zeroes
//    the samples outside the signal when it splits.
// Accumulation order per accumulator is the round-2 kernel's (k-steps group by group, hh, hl, lh
// per step): chroma is bit-identical to it.  LDS: 20 KB ring + 2 x 9 KB images = 38 KB, four
// workgroups (eight waves) per CU; 221 VGPRs, two waves per SIMD.  Rotated timer, one session
// (us per 224 chunks, profiles/r5_cqt_low_variants.txt): round-2 kernel 405.6; this kernel with
// 4 tiles per workgroup and a 4-slot ring 480.9 (16 tile slots for 13.5 tiles of work), 2 tiles
// and a 3-slot ring 416.9 (three workgroups per CU), 2 tiles and 2 slots 358.6.  Probes of the
// last (outputs wrong): no barrier 338.6, no MFMA 259.3, no split 297.5.
// tile geometry knobs (probes; the defaults are the kernel described above).  32-frame tiles, four
// per workgroup (-DC2_FR_=32 -DC2_NW_=4 -DC2_MINB_=3: three waves per SIMD, 168 VGPRs, spills only
// in octave 0's edge instance), bit-identical, round 5, us per 224 chunks (profiles/
// r5_cqt_low_fr32.txt): all three octaves 353.5 against 344.1; octave 0 alone 186.9 against 172.2,
// octave 1 alone 117.7 against 131.3 (134 VGPRs).  Two waves per SIMD (-DC2_MINB_=2) 396.4.  A
// mixed launch (octave 0 at 64 frames, 1-2 at 32) needs two kernels and gives up the octaves'
// overlap inside one launch (all three 328-344 against 424 for the three alone): not built
#ifndef C2_FR_
#define C2_FR_ 64
#endif
#ifndef C2_NW_
#define C2_NW_ 2
#endif
#ifndef C2_MINB_
#define C2_MINB_ 2
#endif
constexpr int C2_FR = C2_FR_;                             // frames per tile (one wave)
constexpr int C2_RT = C2_FR / 16;                         // 16-row tiles per wave
static_assert(C2_RT == 2 || C2_RT == 4, "tile rows");
constexpr int C2_NW = C2_NW_;                             // tiles (waves) per workgroup
constexpr int C2_R = 2;                                   // filter ring slots
constexpr int C2_D = C2_R - 1;                            // slices requested ahead of the step that reads them
constexpr int C2_PS = (CM_NT * 2 + C2_NW - 1) / C2_NW;    // slice DMA pieces per wave per step
#ifndef C2_NRP_
#define C2_NRP_ (C2_FR + 8)
#endif
constexpr int C2_NRP = C2_NRP_;                           // image rows per wave (>= C2_FR + M - 1)
constexpr int C2_IMG = C2_NRP * 64;                       // bytes of one hi (or lo) image
constexpr int C2_RING = C2_R * CM_SLICE * 16;
constexpr int C2_NU = (C2_NRP * 4 + 63) / 64;             // staging rounds (8-sample units per lane)
constexpr int C2_NL = 2 * C2_NU;                          // block loads per wave per group
static_assert(C2_NW * 2 * C2_IMG >= C2_NW * C2_FR * kCqtFilt * 4, "epilogue rows fit the images");
size_t cql_lds_bytes() { return C2_RING + C2_NW * 2 * C2_IMG; }

// image row R keeps its 16-byte piece p (8 halves) at slot p ^ c2_sw(R): every ds_read_b128 lane
// group of an A fragment (rows r..r+15 at pieces 0..3, any r) and every ds_write_b128 group of the
// split (two rows x four pieces) hits distinct banks (checked in tests/test_lds_layout_cpu.py)
__host__ __device__ constexpr int c2_sw(int R) { return ((R >> 2) & 1) << 1; }

__device__ __forceinline__ void c2_ld16(cm_u4& d, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(d) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void c2_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void c2_vmwait_st(cm_u4 (&st)[C2_NL]) {
  static_assert(C2_NL == 10 || C2_NL == 6, "staging registers");
  if constexpr (C2_NL == 10)
    asm volatile("s_waitcnt vmcnt(%10)"
                 : "+v"(st[0]), "+v"(st[1]), "+v"(st[2]), "+v"(st[3]), "+v"(st[4]), "+v"(st[5]), "+v"(st[6]),
                   "+v"(st[7]), "+v"(st[8]), "+v"(st[9])
                 : "i"(N)
                 : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%6)"
                 : "+v"(st[0]), "+v"(st[1]), "+v"(st[2]), "+v"(st[3]), "+v"(st[4]), "+v"(st[5])
                 : "i"(N)
                 : "memory");
}

template <int OCT>
struct C2 {
  static constexpr int H = 512 >> OCT, G = H / 32, M = 1024 / H, NR = C2_FR + M - 1;
  // the block loads of a group are issued at its first step (after that step's slice pieces),
  // and the groups before the last stage the next block
  __host__ __device__ static constexpr bool stage_at(int q, bool last) { return q == 0 && !last; }
  // did step n - j (j >= 1) issue block loads, n at group position q (`last`: the final group)?
  // In the same group: only at position 0 of a group that is not the last; in an earlier group
  // (q < j): at position (q - j) mod M == 0 (an earlier group is never the last)
  __host__ __device__ static constexpr bool staged(int q, int j, bool last) {
    return q >= j ? (q == j && !last) : ((q - j) % M + M) % M == 0;
  }
  // did step n - j issue slice n - j + D (only the last group's final steps do not)?
  __host__ __device__ static constexpr bool sliced(int q, int j, bool last) { return !last || q - j + C2_D < M; }
  // vector-memory operations this wave issued after its pieces of slice n (issued at step n - D)
  // when step n starts: the block loads of steps n - D .. n - 1 and slices n + 1 .. n + D - 1.
  // Steps 0 .. D - 1 over-count (slices 0 .. D - 1 and block 0 were drained in the prologue).
  __host__ __device__ static constexpr int younger(int q, bool last) {
    int y = 0;
    for (int j = 1; j <= C2_D; ++j) y += staged(q, j, last) ? C2_NL : 0;
    for (int j = 1; j < C2_D; ++j) y += sliced(q, j, last) ? C2_PS : 0;
    return y;
  }
};

// vmcnt(younger(q, last)): retires this wave's pieces of slice n (this step's slot).
// C2_SAFE_=1 (probe): vmcnt(0) wherever a block load is younger than the slice
#ifndef C2_SAFE_
#define C2_SAFE_ 0
#endif
// C2_NOBW_=1 (timing probe, outputs wrong): octave C2_NOBW_OCT_ splits its next block without
// waiting for its loads, i.e. the cost of the block loads' exposed latency
#ifndef C2_NOBW_
#define C2_NOBW_ 0
#endif
#ifndef C2_NOBW_OCT_
#define C2_NOBW_OCT_ 0
#endif
template <int OCT, int Q>
__device__ __forceinline__ void c2_wait_slice(bool last) {
  if (C2_SAFE_) {
    if (last) c2_vmwait<C2<OCT>::staged(Q, 1, true) ? 0 : C2<OCT>::younger(Q, true)>();
    else c2_vmwait<C2<OCT>::staged(Q, 1, false) ? 0 : C2<OCT>::younger(Q, false)>();
  } else {
    if (last) c2_vmwait<C2<OCT>::younger(Q, true)>();
    else c2_vmwait<C2<OCT>::younger(Q, false)>();
  }
}

// Block g of this wave's tile into registers: 8-sample unit u = 64 k + lane is row min(u / 4,
// NR - 1), piece u % 4, samples s0 + R H + 32 g + 8 p + [0, 8).  Edge tiles load from clamped
// positions (every load stays inside the signal); c2_split puts the true samples in place.
template <int OCT>
__device__ __forceinline__ void c2_stage(cm_u4 (&st)[C2_NL], const float* y, int64_t s0, int g, int64_t Ly,
                                         bool edge, int lane) {
  using L = C2<OCT>;
#pragma unroll
  for (int k = 0; k < C2_NU; ++k) {
    const int u = 64 * k + lane;
    const int R = min(u >> 2, L::NR - 1), p = u & 3;
    int64_t q = s0 + (int64_t)R * L::H + 32 * g + 8 * p;
    int64_t q1 = q + 4;
    if (edge) {
      q = max((int64_t)0, min(q, Ly - 4));
      q1 = max((int64_t)0, min(q1, Ly - 4));
    }
    c2_ld16(st[2 * k], y + q);
    c2_ld16(st[2 * k + 1], y + q1);
  }
}

// sample q + e of an edge piece loaded from the clamped position b (zero outside [0, Ly))
__device__ __forceinline__ float c2_pick(const cm_u4& v, int64_t q, int e, int64_t Ly) {
  const int64_t b = max((int64_t)0, min(q, Ly - 4));
  const int64_t d = q + e - b;
  const float x = d == 0 ? __uint_as_float(v[0]) : d == 1 ? __uint_as_float(v[1]) : d == 2 ? __uint_as_float(v[2])
                                                                                             : __uint_as_float(v[3]);
  return (q + e >= 0 && q + e < Ly && d >= 0 && d < 4) ? x : 0.0f;
}

// the staged block split into this wave's hi / lo images (rows < NR)
template <int OCT>
__device__ __forceinline__ void c2_split(const cm_u4 (&st)[C2_NL], char* img, float sx, int64_t s0, int g,
                                         int64_t Ly, bool edge, int lane) {
  using L = C2<OCT>;
#pragma unroll
  for (int k = 0; k < C2_NU; ++k) {
    const int u = 64 * k + lane;
    const int R = u >> 2, p = u & 3;
    if (64 * k + 63 >= 4 * L::NR && R >= L::NR) continue;
    float v[8];
    if (edge) {
      const int64_t q = s0 + (int64_t)R * L::H + 32 * g + 8 * p;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = c2_pick(st[2 * k], q, e, Ly);
        v[4 + e] = c2_pick(st[2 * k + 1], q + 4, e, Ly);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = __uint_as_float(st[2 * k][e]);
        v[4 + e] = __uint_as_float(st[2 * k + 1][e]);
      }
    }
    cm_half8 h, l;
    cm_split(v, sx, h, l);
    const int off = R * 64 + 16 * (p ^ c2_sw(R));
    *reinterpret_cast<cm_half8*>(img + off) = h;
    *reinterpret_cast<cm_half8*>(img + C2_IMG + off) = l;
  }
}

template <int OCT, bool EDGE>
__device__ __forceinline__ void cqt_low_tile(const CqmArgs& a, int bx, int c) {
  using L = C2<OCT>;
  constexpr int H = L::H, G = L::G, M = L::M;
  static_assert(G * M == CM_KS && M >= 2 && L::NR <= C2_NRP, "k-step groups");
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* sB = reinterpret_cast<uint4*>(smem);  // [C2_R][CM_SLICE]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // every descriptor read up front, unconditionally: one round trip of scalar loads
  const int T = a.n_frames[c], ti = a.tuning_idx[c], ex = a.oct_ex[c * 7 + OCT];
  const int64_t yoff = OCT == 0 ? a.chunk_off[c] : a.oct_off[c * 7 + OCT], Ly = a.oct_len[c * 7 + OCT];
  if (bx * (C2_NW * C2_FR) >= T) return;
  int t0 = (bx * C2_NW + wave) * C2_FR;
  const bool active = t0 < T;  // an idle tile's wave still issues the DMA, the loads and the barriers
  if (!active) t0 = 0;
  const float* y = (OCT == 0 ? a.sig : a.ws_oct) + yoff;
  const int64_t s0 = (int64_t)t0 * H - 512;
  const bool edge = !(s0 >= 0 && s0 + (int64_t)(C2_FR - 1) * H + kCqtNfft <= Ly);
  if (edge != EDGE) return;  // wave-uniform; both instances issue the same barriers
  const uint4* bsrc = a.bfrag + (size_t)ti * (CM_KS * CM_SLICE);
  char* img = smem + C2_RING + wave * (2 * C2_IMG);
  const float sx = ldexpf(1.0f, ex);
  auto kstep = [](int n) { return n / M + G * (n % M); };
  auto fetch_slice = [&](int n) {
#pragma unroll
    for (int j = 0; j < C2_PS; ++j) {
      int i = wave + C2_NW * j;
      if (i >= CM_NT * 2) i = wave;  // duplicate of this wave's first piece (same bytes, same place)
      cm_dma16(bsrc + kstep(n) * CM_SLICE + i * 64 + lane, sB + (n % C2_R) * CM_SLICE + i * 64);
    }
  };

  // prologue: slices 0-2 in flight, block 0 split, block 1 requested at step 0
  for (int d = 0; d < C2_D; ++d) fetch_slice(d);
  cm_u4 st[C2_NL];
  c2_stage<OCT>(st, y, s0, 0, Ly, EDGE, lane);
  c2_vmwait_st<0>(st);
  if (active) c2_split<OCT>(st, img, sx, s0, 0, Ly, EDGE, lane);

  cm_f4 acc[C2_RT][CM_NT];
#pragma unroll
  for (int rt = 0; rt < C2_RT; ++rt)
#pragma unroll
    for (int nt = 0; nt < CM_NT; ++nt) acc[rt][nt] = cm_f4{0.f, 0.f, 0.f, 0.f};
  const int kp = lane >> 4, rl = lane & 15;
  const uint32_t img_a = lds_addr(img);

  auto step = [&](auto qc, int g, bool last) {
    constexpr int Q = decltype(qc)::value;
    const int n = g * M + Q;
    // retire this wave's pieces of slice n (counted: slices n + 1, n + 2 and the block loads stay
    // in flight); the barrier makes every wave's pieces visible and ends every read of slot
    // (n + 3) % R (step n - 1's)
    c2_wait_slice<OCT, Q>(last);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image writes
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (n + C2_D < CM_KS) fetch_slice(n + C2_D);
    if (L::stage_at(Q, last)) c2_stage<OCT>(st, y, s0, g + 1, Ly, EDGE, lane);
    if (active) {
      // A fragments: rows 16 rt + rl + Q of the image (this wave's own: no barrier guards it)
      const int R = rl + Q;
      const uint32_t aa = img_a + R * 64 + 16 * (kp ^ c2_sw(R));
      const uint32_t sbl = lds_addr(sB + (n % C2_R) * CM_SLICE + lane);
      cm_u4 ah4[C2_RT], al4[C2_RT], b[CM_NT][2];
      static_for<C2_RT>([&](auto rc) { cm_rd<decltype(rc)::value * 1024>(ah4[decltype(rc)::value], aa); });
      static_for<C2_RT>([&](auto rc) { cm_rd<C2_IMG + decltype(rc)::value * 1024>(al4[decltype(rc)::value], aa); });
      cm_rd<0 * 1024>(b[0][0], sbl);
      cm_rd<1 * 1024>(b[0][1], sbl);
      cm_rd<2 * 1024>(b[1][0], sbl);
      cm_rd<3 * 1024>(b[1][1], sbl);
      if constexpr (C2_RT == 4) {
        cm_wait<4>(ah4[0], ah4[1], ah4[2], ah4[3]);  // A + tile 0 landed; tile 1 in flight
        cm_wait<4>(al4[0], al4[1], al4[2], al4[3]);
      } else {
        cm_wait<4>(ah4[0], ah4[1], al4[0], al4[1]);
      }
      cm_half8 ah[C2_RT], al[C2_RT];
#pragma unroll
      for (int rt = 0; rt < C2_RT; ++rt) {
        ah[rt] = __builtin_bit_cast(cm_half8, ah4[rt]);
        al[rt] = __builtin_bit_cast(cm_half8, al4[rt]);
      }
      auto tile = [&](int nt) {
        const cm_half8 bh = __builtin_bit_cast(cm_half8, b[nt][0]);
        const cm_half8 bl = __builtin_bit_cast(cm_half8, b[nt][1]);
#pragma unroll
        for (int rt = 0; rt < C2_RT; ++rt) {
          acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt], bh, acc[rt][nt], 0, 0, 0);
          acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt], bl, acc[rt][nt], 0, 0, 0);
          acc[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[rt], bh, acc[rt][nt], 0, 0, 0);
        }
      };
      // the MFMA cluster at priority 1: the partner wave on the SIMD (another workgroup's tile)
      // takes the VALU / LDS slots around it (round 5: 347.7 -> 339.4 us per 224 chunks, the same
      // pair on cqt_mfma_kernel 328.6 -> 332.1, not kept there; profiles/r5_cqt_sched_variants.txt)
      __builtin_amdgcn_s_setprio(1);
      cm_wait<2>(b[0][0], b[0][1]);
      cm_rd<4 * 1024>(b[2][0], sbl);
      cm_rd<5 * 1024>(b[2][1], sbl);
      tile(0);
      cm_wait<2>(b[1][0], b[1][1]);
      cm_rd<6 * 1024>(b[3][0], sbl);
      cm_rd<7 * 1024>(b[3][1], sbl);
      tile(1);
      cm_wait<2>(b[2][0], b[2][1]);
      cm_rd<8 * 1024>(b[4][0], sbl);
      cm_rd<9 * 1024>(b[4][1], sbl);
      tile(2);
      cm_wait<2>(b[3][0], b[3][1]);
      tile(3);
      cm_wait<0>(b[4][0], b[4][1]);
      tile(4);
      __builtin_amdgcn_s_setprio(0);
    }
    if (Q == M - 1 && !last) {
      // block g + 1 (requested at this group's first step) into the image: every A read of
      // group g is done (their registers were consumed above).  vmcnt(0), not a count: younger
      // slice pieces can retire before the block loads (header).  Splitting after the first or
      // third column tile of the step instead: 351.4 / 350.2 against 347.7 us (round 5)
      if (!(C2_NOBW_ && OCT == C2_NOBW_OCT_)) c2_vmwait_st<0>(st);
      if (active) c2_split<OCT>(st, img, sx, s0, g + 1, Ly, EDGE, lane);
    }
  };
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
    const bool last = g == G - 1;
    static_for<M>([&](auto qc) { step(qc, g, last); });
  }
  if (C2_NOBW_) c2_vmwait<0>();  // (probe) the skipped block waits' loads land before the epilogue
  if (!active) return;
  const int nrow = min(C2_FR, T - t0);
  float* mg = reinterpret_cast<float*>(img);  // [C2_FR][36] rows over this wave's own images
  {
    const float oscale = (float)(1 << (OCT >> 1)) * ((OCT & 1) ? 0x1.6a09e6p+0f : 1.0f);
    const float* isl = a.cqt_isl + ti * kCqtBins + (kCqtBins - kCqtFilt * (OCT + 1));
    const int* bxp = a.bexp + ti * kCqtFilt;
    const int col = lane & 15;
    const float inv0 = ldexpf(1.0f, -(ex + bxp[col])), inv1 = ldexpf(1.0f, -(ex + bxp[16 + col]));
    const float inv2 = ldexpf(1.0f, -(ex + bxp[32 + (col & 3)]));
    const float il0 = isl[col], il1 = isl[16 + col], il2 = isl[32 + (col & 3)];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // this wave's last A reads are done before the rows overlay them
#pragma unroll
    for (int rt = 0; rt < C2_RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int fr = 16 * rt + 4 * (lane >> 4) + i;
        float* m = mg + fr * kCqtFilt;
        m[col] = hypotf(acc[rt][0][i] * inv0 * oscale, acc[rt][1][i] * inv0 * oscale) * il0;
        m[16 + col] = hypotf(acc[rt][2][i] * inv1 * oscale, acc[rt][3][i] * inv1 * oscale) * il1;
        const float im = __shfl_down(acc[rt][4][i], 4, 16);
        if (col < 4) m[32 + col] = hypotf(acc[rt][4][i] * inv2 * oscale, im * inv2 * oscale) * il2;
      }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  float* gp = a.gpart + (a.tf_base[c] + t0) * (7 * 12) + (6 - OCT) * 12;
  for (int qq = lane; qq < nrow * 12; qq += 64) {
    const int fl = qq / 12, cc = qq - 12 * fl;
    const float* m = mg + fl * kCqtFilt;
    gp[fl * (7 * 12) + cc] = cc == 0 ? (m[0] + m[1]) + m[35] : (m[3 * cc - 1] + m[3 * cc]) + m[3 * cc + 1];
  }
}

// CQL_ONLY (timing probe, outputs wrong): >= 0 launches only that octave; 3 (with -DC2_NRP_=80)
// runs octave 3 through this kernel's structure.  Round 5, rotated timer, us per 224 chunks alone
// (profiles/r5_cqt_low_octaves.txt): octave 0 175.2, 1 133.0, 2 116.0, 3 107.7, all three 328.0:
// octave 0 (two k-steps per block, the block loads one k-step ahead of their split) costs most.
// Interleaving the octaves in dispatch order (each XCD's consecutive workgroups the three octaves
// of one tile pair) ran 359.6 -> 392.8 (not kept)
#ifndef CQL_ONLY
#define CQL_ONLY -1
#endif
// C2_XCD_=1 (probe): workgroups dispatched to one XCD (linear ids b, b + 8, ...; placement
// round-robin, speed only) take consecutive (tile pair, chunk, octave) items, so the tiles of one
// (chunk, octave) and their tuning's 320 KB filter set share one L2 instead of seven
#ifndef C2_XCD_
#define C2_XCD_ 0
#endif
__global__ __launch_bounds__(C2_NW * 64, C2_MINB_) void cqt_mfma_low_kernel(CqmArgs a) {
  unsigned bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (C2_XCD_) {
    const unsigned X = gridDim.x, Y = gridDim.y, nb = X * Y * gridDim.z;
    const unsigned b = bx + X * (by + Y * bz), xcd = b & 7, i = b >> 3, q = nb >> 3, rem = nb & 7;
    const unsigned w = xcd < rem ? xcd * (q + 1) + i : rem * (q + 1) + (xcd - rem) * q + i;
    bx = w % X;
    by = (w / X) % Y;
    bz = w / (X * Y);
  }
  const unsigned oz = CQL_ONLY >= 0 ? (unsigned)CQL_ONLY : bz;
  if (oz == 0) {
    cqt_low_tile<0, false>(a, bx, by);
    cqt_low_tile<0, true>(a, bx, by);
  } else if (oz == 1) {
    cqt_low_tile<1, false>(a, bx, by);
    cqt_low_tile<1, true>(a, bx, by);
  } else if (CQL_ONLY != 3) {
    cqt_low_tile<2, false>(a, bx, by);
    cqt_low_tile<2, true>(a, bx, by);
  }
#if CQL_ONLY == 3
  else {
    cqt_low_tile<3, false>(a, bx, by);
    cqt_low_tile<3, true>(a, bx, by);
  }
#endif
}

// Per (chunk, 64-frame tile): chroma = the 7 octave partial rows summed (ascending bins),
// inf-norm per frame, f64 sum over the tile's frames.
__global__ __launch_bounds__(256) void cqt_tail_kernel(const float* gpart, const int64_t* tf_base,
                                                       const int* n_frames, double* partial) {
  __shared__ float sh_ch[CM_FR * 12], sh_nv[CM_FR * 12];
  const int c = blockIdx.y;
  const int T = n_frames[c];
  const int t0 = blockIdx.x * CM_FR;
  if (t0 >= T) return;
  const int nfr = min(CM_FR, T - t0);
  const int tid = threadIdx.x;
  const float* gp = gpart + (tf_base[c] + t0) * (7 * 12);
  for (int q = tid; q < nfr * 12; q += 256) {
    const int fl = q / 12, cc = q - 12 * fl;
    const float* pt = gp + fl * (7 * 12) + cc;
    float ch = 0.0f;
#pragma unroll
    for (int o = 0; o < 7; ++o) ch += pt[12 * o];
    sh_ch[q] = ch;
  }
  __syncthreads();
  for (int q = tid; q < nfr * 12; q += 256) {
    const int fl = q / 12;
    float mx = 0.0f;
    for (int j = 0; j < 12; ++j) mx = fmaxf(mx, fabsf(sh_ch[fl * 12 + j]));
    const double len = (mx < 1.17549435e-38f) ? 1.0 : (double)mx;
    sh_nv[q] = (float)((double)sh_ch[q] / len);
  }
  __syncthreads();
  if (tid < 12) {
    double s = 0.0;
    for (int fl = 0; fl < nfr; ++fl) s += (double)sh_nv[fl * 12 + tid];
    partial[(tf_base[c] / CM_FR + c + blockIdx.x) * 12 + tid] = s;
  }
}

__global__ void chroma_finalize_kernel(const double* partial, const int64_t* tf_base, const int* n_frames, int n,
                                       int fr, float* out_chroma) {
  const int c = blockIdx.x;
  const int k = threadIdx.x;
  if (k >= 12 || c >= n) return;
  const int T = n_frames[c];
  const int nb = (T + fr - 1) / fr;
  const int64_t r0 = tf_base[c] / fr + c;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += partial[(r0 + b) * 12 + k];
  out_chroma[c * 12 + k] = (float)(s / (double)T);
}

// ------------------------------------------------------------------------------ 6. lag
// lag_out[p]: the reference's first argmax over the 12 cyclic lags (f32 dots, compared in
// f64); margin_out[p] (nullable): (best - second best) / |best|, the decision's distance
// from a tie (the soxr_hq -> Kaiser decimator stand-in can move a near-tie)
__global__ void chroma_lag_kernel(const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs,
                                  int* lag_out, double* margin_out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const float* s = chroma + (size_t)src_idx[p] * 12;
  const float* q = chroma + (size_t)nc_idx[p] * 12;
  int best = 0;
  double bv = 0.0, xc[12];
  for (int k = 0; k < 12; ++k) {
    float d = 0.0f;
    for (int j = 0; j < 12; ++j) d = fmaf(s[j], q[(j + k) % 12], d);
    const double v = (double)d;
    xc[k] = v;
    if (k == 0 || v > bv || (v != v && bv == bv)) {
      bv = v;
      best = k;
    }
  }
  lag_out[p] = best > 6 ? best - 12 : best;
  if (margin_out) {
    double second = -INFINITY;
    for (int k = 0; k < 12; ++k)
      if (k != best) second = fmax(second, xc[k]);
    margin_out[p] = bv != 0.0 ? (bv - second) / fabs(bv) : 0.0;
  }
}

// ------------------------------------------------------------------------------ host
struct ChromaWs {
  int64_t* oct_off;
  int64_t* oct_len;
  int* n_frames;
  int* n_tframes;
  int64_t* tf_base;
  int64_t* oct_base;
  float* ws_oct;
  float* peak_pitch;
  float* peak_mag;
  int* chunk_npk;
  double* partial;
  int* tuning_idx;
  float* xmax;  // decimate3 workgroup maxima of |level 0|
  float* gpart; // [tuning frame][7][12] octave chroma partial rows (hybrid CQT)
  int* oct_ex;  // [n][7] f16 split exponents of the CQT operands
};

static inline size_t al256(size_t n) { return (n + 255) & ~(size_t)255; }

size_t chroma_ws_bytes(int n, int64_t total_len) {
  // octave buffers: < total_len * (1/2 + ... ) + padding; tuning frames <= total_len/512 + n
  const int64_t tfr = total_len / 512 + n;
  size_t b = 0;
  b += al256(sizeof(int64_t) * 7 * n) * 2;
  b += al256(sizeof(int) * n) * 4;
  b += al256(sizeof(int64_t) * (n + 1)) * 2;
  b += al256(sizeof(float) * (size_t)(total_len + 64 * 7 * (int64_t)n));
  b += al256(sizeof(float) * (size_t)tfr * kPeakSlots) * 2;
  b += al256(sizeof(double) * (size_t)(tfr / CM_FR + n + 1) * 12);
  b += al256(sizeof(int64_t) * (n + 1));
  b += al256(sizeof(float) * (size_t)(n + (total_len + 64 * 7 * (int64_t)n) / 256 + 2));
  b += al256(sizeof(float) * (size_t)tfr * 84);
  b += al256(sizeof(int) * 7 * n);
  return b + 4096;
}

int launch_chroma_mean(Context& ctx, const float* sig, const int64_t* chunk_off, const int64_t* chunk_len, int n,
                       int64_t total_len, int64_t max_chunk_len, float* out_chroma, float* out_tuning,
                       int* out_tuning_idx, int* out_tuning_margin, const int* tf_skip, int64_t tf_skip_total,
                       float* ext_pitch,
                       float* ext_mag, int* ext_npk, void* wait_event, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n <= 0) return 0;
  const bool ext = ext_pitch && ext_mag && ext_npk;
  if ((tf_skip && !ext) || tf_skip_total < 0) {
    set_error("chroma: tf_skip needs the caller's peak lists (ext_pitch / ext_mag / ext_npk)");
    return -2;
  }
  if (ws_bytes < chroma_ws_bytes(n, total_len)) {
    set_error("chroma: workspace too small");
    return -3;
  }
  if (max_chunk_len <= 0) {
    set_error("chroma: max_chunk_len must be positive");
    return -2;
  }
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* r = p;
    p += al256(bytes);
    return r;
  };
  const int64_t tfr = total_len / 512 + n;
  ChromaWs w;
  w.oct_off = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * 7 * n));
  w.oct_len = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * 7 * n));
  w.n_frames = reinterpret_cast<int*>(take(sizeof(int) * n));
  w.n_tframes = reinterpret_cast<int*>(take(sizeof(int) * n));
  w.chunk_npk = reinterpret_cast<int*>(take(sizeof(int) * n));
  w.tuning_idx = out_tuning_idx ? out_tuning_idx : reinterpret_cast<int*>(take(sizeof(int) * n));
  w.tf_base = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (n + 1)));
  w.oct_base = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (n + 1)));
  w.ws_oct = reinterpret_cast<float*>(take(sizeof(float) * (size_t)(total_len + 64 * 7 * (int64_t)n)));
  w.peak_pitch = reinterpret_cast<float*>(take(sizeof(float) * (size_t)tfr * kPeakSlots));
  w.peak_mag = reinterpret_cast<float*>(take(sizeof(float) * (size_t)tfr * kPeakSlots));
  w.partial = reinterpret_cast<double*>(take(sizeof(double) * (size_t)(tfr / CM_FR + n + 1) * 12));
  int64_t* tp_base = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (n + 1)));
  w.xmax = reinterpret_cast<float*>(take(sizeof(float) * (size_t)(n + (total_len + 64 * 7 * (int64_t)n) / 256 + 2)));
  w.gpart = reinterpret_cast<float*>(take(sizeof(float) * (size_t)tfr * 84));
  w.oct_ex = reinterpret_cast<int*>(take(sizeof(int) * 7 * n));
  if (ext) {  // the caller's lists (zeroed counts): the window stage appends to them too
    w.peak_pitch = ext_pitch;
    w.peak_mag = ext_mag;
    w.chunk_npk = ext_npk;
  }

  {
    MarkSpan ms_(ctx, "chroma_plan", st);
    hipLaunchKernelGGL(chroma_plan_kernel, dim3(1), dim3(256), 0, st, chunk_len, n, w.oct_off, w.oct_len, w.n_frames,
                       w.n_tframes, w.tf_base, w.oct_base, tf_skip, tp_base);
    if (!ext) NC_HIP(hipMemsetAsync(w.chunk_npk, 0, sizeof(int) * n, st));
  }
  // grids are sized by the longest chunk; blocks past a chunk's own length exit.  (Forking
  // the decimation onto a second stream, concurrent with the tuning estimate, measured no
  // gain: the chip is already full with the window chain on the caller's other stream.)
  for (int base = 0; base < 6; base += 3) {
    const int64_t mo = (max_chunk_len >> (base + 3)) + 1;  // >= the longest chunk's level base + 3
    dim3 grid((unsigned)((mo + D3_T - 1) / D3_T), (unsigned)n);
    {
      KTimer kt_(ctx, "decimate", st);
      D3Taps taps;
      std::copy(ctx.t.halfband_f32, ctx.t.halfband_f32 + 2 * kHalfbandK + 1, taps.h);
      for (int rep = 0; rep < NC_PROBE_REPS(3); ++rep)
        hipLaunchKernelGGL(decimate3_kernel, grid, dim3(D3_NT), 0, st, sig, chunk_off, w.oct_off, w.oct_len, w.ws_oct,
                           base, taps, w.xmax, kt_.span());
    }
  }
  PeakArgs pa;
  pa.sig = sig;
  pa.chunk_off = chunk_off;
  pa.chunk_len = chunk_len;
  pa.n_tframes = w.n_tframes;
  pa.tf_base = w.tf_base;
  pa.tp_base = tp_base;
  pa.tf_skip = tf_skip;
  pa.n_chunks = n;
  pa.total_tframes = tfr - tf_skip_total;  // upper bound of tp_base[n]; frames past it are idle
  pa.tw = ctx.t.tw;
  pa.hann2048 = ctx.t.hann2048;
  pa.peak_pitch = w.peak_pitch;
  pa.peak_mag = w.peak_mag;
  pa.chunk_npk = w.chunk_npk;
  {
    const size_t lds = (((TpTw::size + 1) & ~1) + 1024 + (size_t)TP_WAVES * LdsSize<1024>::value) * sizeof(float2);
    const int64_t groups = (pa.total_tframes + TP_WAVES - 1) / TP_WAVES;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(groups, ctx.chroma_cus > 0 ? ctx.chroma_cus : ctx.num_cu));
    {
      KTimer kt_(ctx, "tuning_peaks", st);
      pa.span = kt_.span();
      hipLaunchKernelGGL(tuning_peaks_kernel, dim3(grid), dim3(TP_WAVES * 64), lds, st, pa);
    }
  }
  // the window stage's share of the peaks (tf_skip) must have landed before the select
  if (wait_event) NC_HIP(hipStreamWaitEvent(st, static_cast<hipEvent_t>(wait_event), 0));
  {
    KTimer kt_(ctx, "tuning_select", st);
    OctScale os;
    os.xmax = w.xmax;
    os.oct_off = w.oct_off;
    os.oct_len = w.oct_len;
    os.d3_span = D3_T;
    std::copy(ctx.t.cqm_gpow, ctx.t.cqm_gpow + 7, os.gpow);
    os.oct_ex = w.oct_ex;
    hipLaunchKernelGGL((tuning_select_kernel<TS_NT>), dim3(n), dim3(TS_NT), 0, st, w.peak_pitch, w.peak_mag,
                       w.chunk_npk, w.tf_base, w.tuning_idx, out_tuning, out_tuning_margin, os, kt_.span());
  }
  CqmArgs ma;
  ma.sig = sig;
  ma.chunk_off = chunk_off;
  ma.oct_off = w.oct_off;
  ma.oct_len = w.oct_len;
  ma.n_frames = w.n_frames;
  ma.tuning_idx = w.tuning_idx;
  ma.ws_oct = w.ws_oct;
  ma.tf_base = w.tf_base;
  ma.bfrag = ctx.t.cqm_b;
  ma.bexp = ctx.t.cqm_bexp;
  ma.cqt_isl = ctx.t.cqt_inv_sqrt_len;
  ma.oct_ex = w.oct_ex;
  ma.gpart = w.gpart;
  const int ntile = (int)((1 + max_chunk_len / 512 + CM_FR - 1) / CM_FR);
  {
    // the two CQT kernels are timed apart ("cqt_low", "cqt_high": one rocprof row each); the
    // bench's cqt_chroma unit (7 octaves of every chunk) is their sum
    KTimer kt_(ctx, "cqt_low", st);
    ma.span = kt_.span();
    const int ntl = (int)((1 + max_chunk_len / 512 + C2_FR - 1) / C2_FR);
    const dim3 lg((unsigned)((ntl + C2_NW - 1) / C2_NW), (unsigned)n, CQL_ONLY >= 0 ? 1u : 3u);
    for (int rep = 0; rep < NC_PROBE_REPS(4); ++rep)
      hipLaunchKernelGGL(cqt_mfma_low_kernel, lg, dim3(C2_NW * 64), cql_lds_bytes(), st, ma);
  }
  {
    KTimer kt_(ctx, "cqt_high", st);
    ma.span = kt_.span();
    for (int rep = 0; rep < NC_PROBE_REPS(5); ++rep)
      hipLaunchKernelGGL(cqt_mfma_kernel, dim3((unsigned)((1 + max_chunk_len / 512 + CH_FR - 1) / CH_FR), n),
                         dim3(CM_NTH), cqm_lds_bytes(), st, ma);
  }
  {
    MarkSpan ms_(ctx, "cqt_tail", st);
    hipLaunchKernelGGL(cqt_tail_kernel, dim3(ntile, n), dim3(256), 0, st, w.gpart, w.tf_base, w.n_frames, w.partial);
    hipLaunchKernelGGL(chroma_finalize_kernel, dim3(n), dim3(64), 0, st, w.partial, w.tf_base, w.n_frames, n, CM_FR,
                       out_chroma);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

int launch_chroma_lag(const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs, int* lag_out,
                      double* margin_out, hipStream_t st) {
  if (n_pairs <= 0) return 0;
  hipLaunchKernelGGL(chroma_lag_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, st, chroma, src_idx, nc_idx,
                     n_pairs, lag_out, margin_out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

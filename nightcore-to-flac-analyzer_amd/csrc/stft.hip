// stft.hip — frame-parallel STFT -> power -> Slaney mel -> dB for every frame of
// a batch of sequences (librosa.feature.melspectrogram + power_to_db inside
// onset_strength; oracle/ncref.py mel_db).  Shared by the per-window tempo path
// (hop 512, tempo.py:44 via librosa.onset.onset_strength) and the full-signal
// IBI pass (hop 64, tempo.py:139).
//
// MI355X layout: a workgroup of SM_WAVES waves, one STFT frame per wave (the
// 2048-point real frame is a 1024-point complex wave FFT, radix 16.16.4 through
// an 8.7 KB LDS slot).  Workgroups are persistent and walk a CONTIGUOUS range of
// frames, so the 4x frame overlap (n_fft 2048 / hop 512) is served from the
// XCD's own L2.  Twiddles (2048 entries), the mel CSR weights and their row
// descriptors are staged once per workgroup in LDS.  Per frame the kernel writes
// the 128 dB values, the frame max (the power_to_db top_db clamp needs the
// sequence max) and, optionally, the f64 energy of the hop-length slice the
// frame is centred on (the io.slice_windows energy, io.py:38-40, fused into the
// same HBM read).
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"
#include "nc_piptrack.h"

#include "stft_args.h"

namespace nc {

// Measured and not kept (rounds 2-3): two workgroups per CU (the same alone,
// slower in the step: the extra workgroups queue behind the chroma stream's kernels); the
// mel weights read through L1 instead of LDS (16 waves: 625 against 579 us per 560 windows);
// the Hann window through L1 (607 against 566 us).
constexpr int SM_HANN2 = 1024;  // float2 elements of the staged Hann window
constexpr int SM_WAVES = 14;
constexpr int SM_THREADS = SM_WAVES * 64;
using SmTw = StagedTw<1024>;  // per-stage twiddle table in LDS (conflict-free reads)

// Mel band loops with compile-time trip counts, unrolled in load batches: 562-576 against
// 577-596 us per 560 windows (round 3, same session), bit-identical.
constexpr int kMelJ0 = 3, kMelJ1 = 14;  // float4 steps of the short / long band of a lane (nc_tables.cpp)
constexpr int kMelB = 7;                // steps per load batch

// acc = the fmaf chain of mel_loop over j < nj (< J), in the same order: batches of kMelB
// steps, loads first, then the chain.  Every lane runs all J steps: past its band the weights
// are the table's zero padding, and fmaf(0, p, acc) == acc for the finite p it then reads
// (the power, exchange data, or the slot's zeroed pads), so the sum is bit-identical to the
// per-lane trip count nj, without the 17 exec-masked branches per frame it cost (553 -> 520 us
// per 560 windows, round 3)
template <int J>
__device__ __forceinline__ void mel_unrolled(const float* pw, const float4* w4, int lo, int nj, int lane, float& acc) {
#pragma unroll
  for (int j0 = 0; j0 < J; j0 += kMelB) {
    float4 p[kMelB], w[kMelB];
#pragma unroll
    for (int j = 0; j < kMelB; ++j)
      if (j0 + j < J) {
        p[j] = *reinterpret_cast<const float4*>(pw + lo + 4 * (j0 + j));
        w[j] = w4[(j0 + j) * 64 + lane];
      }
#pragma unroll
    for (int j = 0; j < kMelB; ++j)
      if (j0 + j < J) acc = fmaf(w[j].w, p[j].w, fmaf(w[j].z, p[j].z, fmaf(w[j].y, p[j].y, fmaf(w[j].x, p[j].x, acc))));
  }
}

__device__ __forceinline__ int seq_of_frame(const int64_t* base, int n, int64_t g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (base[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__host__ __device__ __forceinline__ int al4(int n) { return (n + 3) & ~3; }

// mel lane-slot descriptors staged in LDS (a global read at the mel step exposes its latency):
// lo4 | nj4 << 11 | band << 16 per (slot, lane)
constexpr int SM_MT = 128;
__host__ __device__ __forceinline__ int mel_pack(int lo4, int nj4, int band) { return lo4 | (nj4 << 11) | (band << 16); }

size_t stft_mel_lds_bytes(int mel_j) {
  return (size_t)al4(SmTw::size) * sizeof(float2) + (size_t)mel_j * 64 * sizeof(float4) +
         (size_t)SM_HANN2 * sizeof(float2) + (size_t)SM_MT * sizeof(int) +
         (size_t)SM_WAVES * LdsSize<1024>::value * sizeof(float2);
}

__global__ __launch_bounds__(SM_THREADS) void stft_mel_kernel(StftMelArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* sh_tw = reinterpret_cast<float2*>(smem);
  float4* sh_w4 = reinterpret_cast<float4*>(sh_tw + al4(SmTw::size));  // [mel_j0 + mel_j1][64]
  const int lane0 = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  float2* sh_hann = reinterpret_cast<float2*>(sh_w4 + (a.mel_j0 + a.mel_j1) * 64);
  int* sh_mt = reinterpret_cast<int*>(sh_hann + SM_HANN2);
  float2* fftbuf = reinterpret_cast<float2*>(sh_mt + SM_MT) + wave * LdsSize<1024>::value;

  fill_staged_tw<1024>(sh_tw, a.tw, threadIdx.x, SM_THREADS);
  for (int i = threadIdx.x; i < SM_HANN2; i += SM_THREADS) sh_hann[i] = reinterpret_cast<const float2*>(a.hann2048)[i];
  for (int i = threadIdx.x; i < (a.mel_j0 + a.mel_j1) * 64; i += SM_THREADS) sh_w4[i] = a.mel_w4[i];
  if (threadIdx.x < SM_MT) sh_mt[threadIdx.x] = mel_pack(a.mel_lo4[threadIdx.x], a.mel_nj4[threadIdx.x], a.mel_band[threadIdx.x]);
  const float4* mw4 = sh_w4;
  // the wave's slot zeroed once: the pad elements of the exchange layout are never written, and
  // the mel steps past a band's end read them (times a zero weight)
  for (int i = threadIdx.x & 63; i < LdsSize<1024>::value; i += 64) fftbuf[i] = make_float2(0.f, 0.f);
  __syncthreads();

  const int64_t n_groups = (a.total_frames + SM_WAVES - 1) / SM_WAVES;
  const int64_t gb = n_groups * blockIdx.x / gridDim.x, ge = n_groups * (blockIdx.x + 1) / gridDim.x;
  // The wave's frames g = grp * SM_WAVES + wave rise by SM_WAVES: their sequence is tracked
  // forward, its bounds, flags, length and offset reloaded only when g crosses into a later
  // sequence, instead of a 64-bit division or binary search and dependent loads per frame
  int s = -1;
  int64_t sb = 0, se = -1, t0 = 0, L = 0, off = 0;
  int wc = -1;  // the 20 s chunk the sequence starts (shared tuning frames), or -1
  bool act = true;
  for (int64_t grp = gb; grp < ge; ++grp) {
    const int64_t g = grp * SM_WAVES + wave;
    if (g >= a.total_frames) break;
    if (g >= se) {
      if (s < 0) {
        s = a.frame_base ? seq_of_frame(a.frame_base, a.n_seq, g) : (int)(g / a.uniform_T);
      } else if (a.frame_base) {
        do ++s;
        while (s + 1 < a.n_seq && a.frame_base[s + 1] <= g);
      } else {
        s = (int)(g / a.uniform_T);
      }
      s = uniform32(s);
      sb = uniform64(a.frame_base ? a.frame_base[s] : (int64_t)s * a.uniform_T);
      se = uniform64(a.frame_base ? (s + 1 < a.n_seq ? a.frame_base[s + 1] : INT64_MAX) : sb + a.uniform_T);
      t0 = uniform64(a.frame_base && a.seq_t0 ? a.seq_t0[s] : 0);
      act = !a.active || a.active[s];
      L = uniform64(a.seq_len ? a.seq_len[s] : a.uniform_len);
      off = uniform64(a.seq_off[s]);
      wc = uniform32(a.win_chunk ? a.win_chunk[s] : -1);
    }
    if (!act) continue;
    const int64_t t = g - sb + t0;
    const float* x = a.sig + off;
    const int64_t s0 = t * a.hop - 1024;

    // Opaque lane id: every per-lane address and table load is recomputed each
    // frame instead of being hoisted out of the loop (which would cost occupancy).
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int jin = fft_in_lane(lane);  // this lane's stage-1 butterfly: samples x[2 (jin + 64 r)]
    const float2* twl = sh_tw;
    const float* hann = a.hann2048;
    FftIn<1024> in;
    double e = 0.0;
    const bool interior = s0 >= 0 && s0 + 2048 <= L;
    if (interior) {
      float2 xv[16], hw[16];  // samples and window pairs (h[2n], h[2n + 1]), n = lane + 64 r
      if ((off & 1) == 0) {
        const float2* x2 = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
        for (int r = 0; r < 16; ++r) xv[r] = x2[jin + 64 * r];  // issued first: the LDS batch hides under them
      } else {
        // a sequence at an odd sample (a trimmed file starts anywhere): the pairs are not 8-byte
        // aligned, so two dword loads each, still without bounds tests (round 3: the per-sample
        // edge path used to take these frames, +45 % on stft_mel)
        const float* xs = x + s0;
#pragma unroll
        for (int r = 0; r < 16; ++r) xv[r] = make_float2(xs[2 * (jin + 64 * r)], xs[2 * (jin + 64 * r) + 1]);
      }
      lds_read16_strided<0, 64 * 8>(hw, lds_addr(sh_hann + jin));
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = jin + 64 * r;
        const float2 v = xv[r];
        const float2 h = hw[r];
        if (r >= 8 && r < 12) {
          // the hop slice's samples, selected instead of branched on (fma(0, 0, e) == e)
          const bool in_hop = 2 * n - 1024 < a.hop;
          const double dx = in_hop ? (double)v.x : 0.0, dy = in_hop ? (double)v.y : 0.0;
          e = fma(dx, dx, e);
          e = fma(dy, dy, e);
        }
        in[0][r] = make_float2(v.x * h.x, v.y * h.y);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = jin + 64 * r;
        const int64_t i0 = s0 + 2 * n;
        const float x0 = (i0 >= 0 && i0 < L) ? x[i0] : 0.0f;
        const float x1 = (i0 + 1 >= 0 && i0 + 1 < L) ? x[i0 + 1] : 0.0f;
        if (r >= 8 && r < 12) {
          const int q = 2 * n - 1024;
          if (q < a.hop) {
            e = fma((double)x0, (double)x0, e);
            e = fma((double)x1, (double)x1, e);
          }
        }
        in[0][r] = make_float2(x0 * hann[2 * n], x1 * hann[2 * n + 1]);
      }
    }
    if (a.frame_energy) {
      e = wave_sum_u(e);
      if (lane == 0) a.frame_energy[g] = e;
    }
    // 1024-point complex FFT of the packed frame: stages 1-2 through LDS, the last stage on
    // mirror-paired butterflies, then the real split and |X|^2 straight from registers
    stockham_stage_regs<1024, 16, 1, 64, false, 0, 0>(in, fftbuf, twl, jin);
    stockham_stage<1024, 16, 16, 64, false, 0, 0>(fftbuf, twl, lane);
    float2 v[4][4];
    fft1024_last_mirror<SmTw::s3, true>(fftbuf, twl, lane, v);
    // power |2 X[k]|^2 = 4 P[k], k in [0, 1024] (the split without its 0.5 scalings, exact; the mel
    // weights carry the 0.25), over the FFT slot (all Z reads precede)
    float* pw = reinterpret_cast<float*>(fftbuf);
    // a leading frame of a window that starts a 20 s chunk is also that chunk's tuning frame
    // t (same samples, padding and FFT): estimate_tuning's piptrack runs here, on the same
    // 2|X| values tuning_peaks_kernel computes (nc_piptrack.h; its decisions are scale-free): the
    // frame max from the split's registers, the stencil bins' 2|X| beside the power (which the
    // mel step needs)
    if (wc >= 0 && t < a.tp_frames) {
      float pmax = 0.0f;
      rsplit_mirror<SmTw::split, false>(v, twl, lane, [&](int k, float2 X, float2 XN) {
        const float p1 = fmaf(X.x, X.x, X.y * X.y), p2 = fmaf(XN.x, XN.x, XN.y * XN.y);
        pw[k] = p1;
        pw[1024 - k] = p2;
        pmax = fmaxf(pmax, fmaxf(p1, p2));
      });
      const float mx = __fsqrt_rn(wave_max_u(pmax));
      float* mg = pw + kPipMag;  // |X[k]| at mg[k - (kPipLo - 1)]
#pragma unroll
      for (int q = 0; q < (kPipHi - kPipLo + 3 + 63) / 64; ++q) {
        const int k = kPipLo - 1 + 64 * q + lane;
        if (64 * (q + 1) <= kPipHi - kPipLo + 3 || k <= kPipHi + 1)  // test the last round only
          mg[k - (kPipLo - 1)] = __fsqrt_rn(pw[k]);
      }
      const int64_t base = uniform64(a.chunk_tf_base[wc]) * kPeakSlots;
      piptrack_append([&](int k) { return mg[k - (kPipLo - 1)]; }, mx, lane, &a.chunk_npk[wc], a.peak_pitch + base,
                      a.peak_mag + base, reinterpret_cast<int*>(pw + kPipKpk));
    } else {
      rsplit_mirror<SmTw::split, false>(v, twl, lane, [&](int k, float2 X, float2 XN) {
        pw[k] = fmaf(X.x, X.x, X.y * X.y);
        pw[1024 - k] = fmaf(XN.x, XN.x, XN.y * XN.y);
      });
    }
    // Slaney mel: lane l owns one short and one long band (mel_band: spread over the lanes so
    // the float4 power reads are bank-conflict free), read as float4 steps from a 16-byte
    // aligned first bin with zero-padded weights (fmaf chain in bin order, as the CSR form)
    float acc0 = 0.0f, acc1 = 0.0f;
    const int mt0 = sh_mt[lane], mt1 = sh_mt[64 + lane];
    mel_unrolled<kMelJ0>(pw, mw4, mt0 & 2047, (mt0 >> 11) & 31, lane, acc0);
    mel_unrolled<kMelJ1>(pw, mw4 + kMelJ0 * 64, mt1 & 2047, (mt1 >> 11) & 31, lane, acc1);
    const float db0 = 10.0f * log10f(fmaxf(1e-10f, acc0));
    const float db1 = 10.0f * log10f(fmaxf(1e-10f, acc1));
    float* row = a.sdb + g * 128;
    row[mt0 >> 16] = db0;
    row[mt1 >> 16] = db1;
    const float mx = wave_max_u(fmaxf(db0, db1));
    if (lane == 0) a.frame_max[g] = mx;
  }
}

int launch_stft_mel(Context& ctx, const StftMelArgs& args, hipStream_t st) {
  if (args.total_frames <= 0) return 0;
  StftMelArgs a = args;
  a.tw = ctx.t.tw;
  a.hann2048 = ctx.t.hann2048;
  a.mel_lo = ctx.t.mel_lo;
  a.mel_len = ctx.t.mel_len;
  a.mel_off = ctx.t.mel_off;
  a.mel_w = ctx.t.mel_w;
  a.mel_nnz = ctx.t.mel_nnz;
  a.mel_w4 = ctx.t.mel_w4;
  a.mel_lo4 = ctx.t.mel_lo4;
  a.mel_nj4 = ctx.t.mel_nj4;
  a.mel_band = ctx.t.mel_band;
  a.mel_j0 = ctx.t.mel_j0;
  a.mel_j1 = ctx.t.mel_j1;
  if (a.hop <= 0 || a.hop > 512 || (a.hop & 1)) {
    set_error("stft_mel: hop must be even and <= 512");
    return -2;
  }
  if (a.mel_j0 != kMelJ0 || a.mel_j1 != kMelJ1) {
    set_error("stft_mel: mel table trip counts differ from the kernel's compile-time ones");
    return -2;
  }
  const size_t lds = stft_mel_lds_bytes(a.mel_j0 + a.mel_j1);
  if (lds > 160 * 1024) {
    set_error("stft_mel: LDS layout exceeds 160 KiB");
    return -2;
  }
  const int64_t n_groups = (a.total_frames + SM_WAVES - 1) / SM_WAVES;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(n_groups, (int64_t)ctx.num_cu * (lds <= 80 * 1024 ? 2 : 1)));
  {
    KTimer kt_(ctx, "stft_mel", st);
    a.span = kt_.span();
    hipLaunchKernelGGL(stft_mel_kernel, dim3(grid), dim3(SM_THREADS), lds, st, a);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

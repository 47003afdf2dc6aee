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
//   1. decimate_kernel x6     y_{i+1} = sqrt(2) * halfband(y_i)[::2]  (soxr_hq replacement)
//   2. tuning_peaks_kernel    STFT 2048/512 (Hann) -> piptrack peaks per frame (fixed slots)
//   3. tuning_select_kernel   median(mag) -> residual histogram (0.01 bins) -> tuning index
//   4. cqt_chroma_kernel      7 waves = 7 octaves of one frame: rect-window FFT 1024 ->
//                             sparse basis[tuning] -> |C|/sqrt(len) -> 12-bin chroma ->
//                             inf-norm -> per-block partial sums (f64)
//   5. chroma_finalize_kernel mean over frames -> f32[12] per chunk
//   6. chroma_lag_kernel      argmax_k dot(src, roll(nc, -k)), wrapped to [-5, 6]
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

constexpr int kPeakSlots = 192;  // >= max piptrack peaks per frame (bins 14..371 -> <= 179)

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

__global__ void chroma_plan_kernel(const int64_t* chunk_len, int n, int64_t* oct_off, int64_t* oct_len,
                                   int* n_frames, int* n_tframes, int64_t* tf_base) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t acc = 0, tacc = 0;
  for (int c = 0; c < n; ++c) {
    int64_t L = chunk_len[c];
    int hop = 512;
    int tmin = 0x7fffffff;
    for (int i = 0; i < 7; ++i) {
      oct_len[c * 7 + i] = L;
      if (i == 0) oct_off[c * 7 + i] = -1;
      else {
        oct_off[c * 7 + i] = acc;
        acc += (L + 63) & ~63LL;
      }
      tmin = min(tmin, (int)(1 + L / hop));
      hop >>= 1;
      L = (L + 1) / 2;
    }
    n_frames[c] = tmin;
    n_tframes[c] = (int)(1 + chunk_len[c] / 512);
    tf_base[c] = tacc;
    tacc += n_tframes[c];
  }
  tf_base[n] = tacc;
}

// ------------------------------------------------------------------------------ 1. decimation
__global__ __launch_bounds__(256) void decimate_kernel(const float* sig, const int64_t* chunk_off,
                                                       const int64_t* oct_off, const int64_t* oct_len,
                                                       float* ws_oct, int level, const double* taps,
                                                       int K, int64_t max_out) {
  const int c = blockIdx.y;
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t Lin = oct_len[c * 7 + level];
  const int64_t Lout = oct_len[c * 7 + level + 1];
  if (m >= Lout) return;
  const float* in = level == 0 ? sig + chunk_off[c] : ws_oct + oct_off[c * 7 + level];
  float* out = ws_oct + oct_off[c * 7 + level + 1];
  double acc = 0.0;
  for (int j = 0; j <= 2 * K; ++j) {
    const double h = taps[j];
    if (h == 0.0) continue;
    const int64_t i = 2 * m - (j - K);
    if (i >= 0 && i < Lin) acc += h * (double)in[i];
  }
  out[m] = (float)(acc * 1.4142135623730951);
}

// ------------------------------------------------------------------------------ 2. tuning peaks
struct PeakArgs {
  const float* sig;
  const int64_t* chunk_off;
  const int64_t* chunk_len;
  const int* n_tframes;
  const int64_t* tf_base;
  int n_chunks;
  int64_t total_tframes;
  const float2* tw;
  const float* hann2048;
  float* peak_pitch;  // [total_tframes][kPeakSlots]
  float* peak_mag;
  int* peak_cnt;      // [total_tframes]
};

__global__ __launch_bounds__(256) void tuning_peaks_kernel(PeakArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float2* fftbuf = reinterpret_cast<float2*>(smem) + wave * LdsSize<1024>::value;
  const int64_t gf = (int64_t)blockIdx.x * 4 + wave;
  if (gf >= a.total_tframes) return;
  int lo = 0, hi = a.n_chunks - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.tf_base[mid] <= gf) lo = mid;
    else hi = mid - 1;
  }
  const int c = lo;
  const int t = (int)(gf - a.tf_base[c]);
  if (t >= a.n_tframes[c]) return;
  const float* x = a.sig + a.chunk_off[c];
  const int64_t L = a.chunk_len[c];
  const int64_t s0 = (int64_t)t * 512 - 1024;
  FftIn<1024> in;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = lane + 64 * r;
    const int64_t i0 = s0 + 2 * n;
    const float x0 = (i0 >= 0 && i0 < L) ? x[i0] : 0.0f;
    const float x1 = (i0 + 1 >= 0 && i0 + 1 < L) ? x[i0 + 1] : 0.0f;
    in[0][r] = make_float2(x0 * a.hann2048[2 * n], x1 * a.hann2048[2 * n + 1]);
  }
  wave_fft<1024>(in, fftbuf, a.tw, lane);
  float m1[9], m2[9];
#pragma unroll
  for (int m = 0; m < 9; ++m) {
    const int k = lane + 64 * m;
    if (k <= 512) {
      float2 X, XN;
      rfft_split(fftbuf, a.tw, 1024, k, X, XN);
      m1[m] = hypotf(X.x, X.y);
      m2[m] = hypotf(XN.x, XN.y);
    }
  }
  float* S = reinterpret_cast<float*>(fftbuf);
#pragma unroll
  for (int m = 0; m < 9; ++m) {
    const int k = lane + 64 * m;
    if (k <= 512) {
      S[k] = m1[m];
      S[1024 - k] = m2[m];
    }
  }
  // frame max over all 1025 bins
  float mx = 0.0f;
  for (int k = lane; k <= 1024; k += 64) mx = fmaxf(mx, S[k]);
  mx = wave_max(mx);
  const float ref = 0.1f * mx;
  // bins inside [150, 4000) Hz: k*22050/2048 -> 14..371
  const int klo = 14, khi = 371;
  int base = 0;
  for (int k0 = klo; k0 <= khi; k0 += 64) {
    const int k = k0 + lane;
    bool pk = false;
    float pitch = 0.0f, mag = 0.0f;
    if (k <= khi) {
      const float sm = S[k - 1], s = S[k], sp = S[k + 1];
      const float zm = sm > ref ? sm : 0.0f, z = s > ref ? s : 0.0f, zp = sp > ref ? sp : 0.0f;
      pk = (z > zm) && (z >= zp);
      if (pk) {
        // parabolic shift (librosa numba stencil, f64 arithmetic, stored f32)
        const double aa = (double)(sp + sm) - 2.0 * (double)s;  // f32 add, then f64 (numba typing)
        const double bb = (double)(sp - sm) / 2.0;
        const float shift = (fabs(bb) >= fabs(aa)) ? 0.0f : (float)(-bb / aa);
        const float avg = (sp - sm) / 2.0f;
        const float dskew = (0.5f * avg) * shift;
        pitch = (float)((((double)k + (double)shift) * 22050.0) / 2048.0);
        mag = s + dskew;
      }
    }
    const unsigned long long bal = __ballot(pk);
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    if (pk && base + rank < kPeakSlots) {
      a.peak_pitch[gf * kPeakSlots + base + rank] = pitch;
      a.peak_mag[gf * kPeakSlots + base + rank] = mag;
    }
    base += __popcll(bal);
  }
  if (lane == 0) a.peak_cnt[gf] = min(base, kPeakSlots);
}

// ------------------------------------------------------------------------------ 3. tuning select
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

template <int NT>
__global__ __launch_bounds__(NT) void tuning_select_kernel(const float* peak_pitch, const float* peak_mag,
                                                           const int* peak_cnt, const int* n_tframes,
                                                           const int64_t* tf_base, int* tuning_idx,
                                                           float* tuning_val) {
  __shared__ BlockScratch<NT> bs;
  __shared__ int hist[256];
  __shared__ int counts[100];
  const int c = blockIdx.x;
  const int64_t f0 = tf_base[c];
  const int T = n_tframes[c];
  // total peaks
  int tot = 0;
  for (int t = threadIdx.x; t < T; t += NT) tot += peak_cnt[f0 + t];
  tot = block_sum_i<NT>(tot, bs);
  // median of mags (all peaks have pitch > 0)
  float thr = 0.0f;
  if (tot > 0) {
    // radix select over f32 keys (32 bits, 4 passes of 8 bits)
    auto fkey = [](float f) {
      unsigned u = __float_as_uint(f);
      return (u >> 31) ? ~u : (u | 0x80000000u);
    };
    auto kth = [&](int k) {
      unsigned prefix = 0, mask = 0;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0;
        __syncthreads();
        for (int t = 0; t < T; ++t) {
          const int n = peak_cnt[f0 + t];
          for (int j = threadIdx.x; j < n; j += NT) {
            const unsigned key = fkey(peak_mag[(f0 + t) * kPeakSlots + j]);
            if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
          }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          int kk = k, d = 0;
          for (; d < 256; ++d) {
            if (kk < hist[d]) break;
            kk -= hist[d];
          }
          bs.i[0] = d;
          bs.i[1] = kk;
        }
        __syncthreads();
        prefix |= (unsigned)bs.i[0] << shift;
        mask |= 255u << shift;
        k = bs.i[1];
        __syncthreads();
      }
      const unsigned u = (prefix >> 31) ? (prefix & 0x7fffffffu) : ~prefix;
      return __uint_as_float(u);
    };
    if (tot & 1) thr = kth(tot / 2);
    else {
      const float lo = kth(tot / 2 - 1), hi = kth(tot / 2);
      thr = (lo + hi) / 2.0f;
    }
  }
  for (int i = threadIdx.x; i < 100; i += NT) counts[i] = 0;
  __syncthreads();
  int nsel = 0;
  for (int t = 0; t < T; ++t) {
    const int n = peak_cnt[f0 + t];
    for (int j = threadIdx.x; j < n; j += NT) {
      const float mg = peak_mag[(f0 + t) * kPeakSlots + j];
      const float p = peak_pitch[(f0 + t) * kPeakSlots + j];
      if (mg >= thr && p > 0.0f) {
        const float o = log2f(p / 27.5f);
        float r = fmodf(36.0f * o, 1.0f);
        if (r < 0.0f) r += 1.0f;
        if (r >= 0.5f) r -= 1.0f;
        atomicAdd(&counts[tuning_bin(r)], 1);
        ++nsel;
      }
    }
  }
  nsel = block_sum_i<NT>(nsel, bs);
  if (threadIdx.x == 0) {
    int best = 50;
    if (nsel > 0) {
      best = 0;
      for (int j = 1; j < 100; ++j)
        if (counts[j] > counts[best]) best = j;
    }
    tuning_idx[c] = best;
    tuning_val[c] = (float)((double)best * (1.0 / 100.0) + (-0.5));
  }
}

// ------------------------------------------------------------------------------ 4. CQT + chroma
struct CqtArgs {
  const float* sig;
  const int64_t* chunk_off;
  const int64_t* oct_off;
  const int64_t* oct_len;
  const int* n_frames;
  const int* tuning_idx;
  const float* ws_oct;
  int nblk;
  const float2* tw;
  const int* cqt_lo;
  const int* cqt_len;
  const int* cqt_off;
  const float2* cqt_w;
  const float* cqt_isl;
  double* partial;  // [n][nblk][12]
};

constexpr int CQ_WAVES = 7;

__global__ __launch_bounds__(CQ_WAVES * 64) void cqt_chroma_kernel(CqtArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, oct = threadIdx.x >> 6;
  const int c = blockIdx.y, blk = blockIdx.x;
  float2* fftbuf = reinterpret_cast<float2*>(smem) + oct * LdsSize<512>::value;
  float* row = reinterpret_cast<float*>(reinterpret_cast<float2*>(smem) + CQ_WAVES * LdsSize<512>::value);
  const int T = a.n_frames[c];
  const int ti = a.tuning_idx[c];
  const float* y = oct == 0 ? a.sig + a.chunk_off[c] : a.ws_oct + a.oct_off[c * 7 + oct];
  const int64_t Ly = a.oct_len[c * 7 + oct];
  const int hop = 512 >> oct;
  const float oscale = sqrtf((float)(1 << oct));  // fft_basis *= sqrt(sr / my_sr)
  double acc = 0.0;                               // lanes 0..11 of wave 0: chroma sums
  for (int t = blk; t < T; t += a.nblk) {
    const int64_t s0 = (int64_t)t * hop - 512;
    FftIn<512> in;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int n = lane + 64 * r;
      const int64_t i0 = s0 + 2 * n;
      const float x0 = (i0 >= 0 && i0 < Ly) ? y[i0] : 0.0f;
      const float x1 = (i0 + 1 >= 0 && i0 + 1 < Ly) ? y[i0 + 1] : 0.0f;
      in[0][r] = make_float2(x0, x1);
    }
    wave_fft<512>(in, fftbuf, a.tw, lane);
    float2 d1[5], d2[5];
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int k = lane + 64 * m;
      if (k <= 256) rfft_split(fftbuf, a.tw, 512, k, d1[m], d2[m]);
    }
    float2* D = fftbuf;  // reuse as D[0..512] unpadded
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int k = lane + 64 * m;
      if (k <= 256) {
        D[k] = d1[m];
        D[512 - k] = d2[m];
      }
    }
    // 36 filters: lanes 0..35
    if (lane < kCqtFilt) {
      const int fi = ti * kCqtFilt + lane;
      const int lo = a.cqt_lo[fi], len = a.cqt_len[fi], off = a.cqt_off[fi];
      float re = 0.0f, im = 0.0f;
      for (int j = 0; j < len; ++j) {
        const float2 w = a.cqt_w[off + j];
        const float2 d = D[lo + j];
        re = fmaf(w.x, d.x, fmaf(-w.y, d.y, re));
        im = fmaf(w.x, d.y, fmaf(w.y, d.x, im));
      }
      const int bin = kCqtBins - kCqtFilt * (oct + 1) + lane;
      row[bin] = hypotf(re * oscale, im * oscale) * a.cqt_isl[ti * kCqtBins + bin];
    }
    __syncthreads();
    if (oct == 0) {
      // chroma c <- CQT bins with (j mod 36) in {3c-1, 3c, 3c+1} (mod 36), ascending j
      float ch = 0.0f;
      if (lane < 12) {
        // 3 bins per chroma per octave, octave-major, ascending within the octave
        for (int o = 0; o < 7; ++o) {
          const int b = 36 * o;
          if (lane == 0) {
            ch += row[b];
            ch += row[b + 1];
            ch += row[b + 35];
          } else {
            ch += row[b + 3 * lane - 1];
            ch += row[b + 3 * lane];
            ch += row[b + 3 * lane + 1];
          }
        }
      }
      float mx = (lane < 12) ? fabsf(ch) : 0.0f;
      mx = wave_max(mx);
      const double len = (mx < 1.17549435e-38f) ? 1.0 : (double)mx;
      if (lane < 12) acc += (double)(float)((double)ch / len);
    }
    __syncthreads();
  }
  if (oct == 0 && lane < 12) a.partial[((size_t)c * a.nblk + blk) * 12 + lane] = acc;
}

__global__ void chroma_finalize_kernel(const double* partial, int nblk, const int* n_frames, int n,
                                       float* out_chroma) {
  const int c = blockIdx.x;
  const int k = threadIdx.x;
  if (k >= 12 || c >= n) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += partial[((size_t)c * nblk + b) * 12 + k];
  out_chroma[c * 12 + k] = (float)(s / (double)n_frames[c]);
}

// ------------------------------------------------------------------------------ 6. lag
__global__ void chroma_lag_kernel(const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs,
                                  int* lag_out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const float* s = chroma + (size_t)src_idx[p] * 12;
  const float* q = chroma + (size_t)nc_idx[p] * 12;
  int best = 0;
  double bv = 0.0;
  for (int k = 0; k < 12; ++k) {
    float d = 0.0f;
    for (int j = 0; j < 12; ++j) d = fmaf(s[j], q[(j + k) % 12], d);
    const double v = (double)d;
    if (k == 0 || v > bv || (v != v && bv == bv)) {
      bv = v;
      best = k;
    }
  }
  lag_out[p] = best > 6 ? best - 12 : best;
}

// ------------------------------------------------------------------------------ host
struct ChromaWs {
  int64_t* oct_off;
  int64_t* oct_len;
  int* n_frames;
  int* n_tframes;
  int64_t* tf_base;
  float* ws_oct;
  float* peak_pitch;
  float* peak_mag;
  int* peak_cnt;
  double* partial;
  int* tuning_idx;
};

static inline size_t al256(size_t n) { return (n + 255) & ~(size_t)255; }

constexpr int kCqtBlk = 32;  // frame blocks per chunk

size_t chroma_ws_bytes(int n, int64_t total_len) {
  // octave buffers: < total_len * (1/2 + ... ) + padding; tuning frames <= total_len/512 + n
  const int64_t tfr = total_len / 512 + n;
  size_t b = 0;
  b += al256(sizeof(int64_t) * 7 * n) * 2;
  b += al256(sizeof(int) * n) * 3;
  b += al256(sizeof(int64_t) * (n + 1));
  b += al256(sizeof(float) * (size_t)(total_len + 64 * 7 * (int64_t)n));
  b += al256(sizeof(float) * (size_t)tfr * kPeakSlots) * 2;
  b += al256(sizeof(int) * (size_t)tfr);
  b += al256(sizeof(double) * (size_t)n * kCqtBlk * 12);
  return b + 4096;
}

int launch_chroma_mean(Context& ctx, const float* sig, const int64_t* chunk_off, const int64_t* chunk_len, int n,
                       int64_t total_len, int64_t max_chunk_len, float* out_chroma, float* out_tuning, int* out_tuning_idx, void* ws,
                       size_t ws_bytes, hipStream_t st) {
  if (n <= 0) return 0;
  if (ws_bytes < chroma_ws_bytes(n, total_len)) {
    set_error("chroma: workspace too small");
    return -3;
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
  w.tuning_idx = out_tuning_idx ? out_tuning_idx : reinterpret_cast<int*>(take(sizeof(int) * n));
  w.tf_base = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (n + 1)));
  w.ws_oct = reinterpret_cast<float*>(take(sizeof(float) * (size_t)(total_len + 64 * 7 * (int64_t)n)));
  w.peak_pitch = reinterpret_cast<float*>(take(sizeof(float) * (size_t)tfr * kPeakSlots));
  w.peak_mag = reinterpret_cast<float*>(take(sizeof(float) * (size_t)tfr * kPeakSlots));
  w.peak_cnt = reinterpret_cast<int*>(take(sizeof(int) * (size_t)tfr));
  w.partial = reinterpret_cast<double*>(take(sizeof(double) * (size_t)n * kCqtBlk * 12));

  hipLaunchKernelGGL(chroma_plan_kernel, dim3(1), dim3(64), 0, st, chunk_len, n, w.oct_off, w.oct_len, w.n_frames,
                     w.n_tframes, w.tf_base);
  // host-side bound for grids: longest chunk
  // (grid.x sized by total_len, threads beyond a chunk's length exit)
  const int64_t max_chunk = max_chunk_len;
  for (int lvl = 0; lvl < 6; ++lvl) {
    const int64_t mo = (max_chunk >> (lvl + 1)) + 1;
    dim3 grid((unsigned)((mo + 255) / 256), (unsigned)n);
    hipLaunchKernelGGL(decimate_kernel, grid, dim3(256), 0, st, sig, chunk_off, w.oct_off, w.oct_len, w.ws_oct,
                       lvl, ctx.t.halfband, kHalfbandK, mo);
  }
  PeakArgs pa;
  pa.sig = sig;
  pa.chunk_off = chunk_off;
  pa.chunk_len = chunk_len;
  pa.n_tframes = w.n_tframes;
  pa.tf_base = w.tf_base;
  pa.n_chunks = n;
  pa.total_tframes = tfr;  // upper bound; frames beyond tf_base[n] are skipped below
  pa.tw = ctx.t.tw;
  pa.hann2048 = ctx.t.hann2048;
  pa.peak_pitch = w.peak_pitch;
  pa.peak_mag = w.peak_mag;
  pa.peak_cnt = w.peak_cnt;
  // exact total tuning frames = sum(1 + len/512) <= tfr; extra waves find t >= n_tframes
  hipLaunchKernelGGL(tuning_peaks_kernel, dim3((unsigned)((tfr + 3) / 4)), dim3(256),
                     4 * LdsSize<1024>::value * sizeof(float2), st, pa);
  hipLaunchKernelGGL((tuning_select_kernel<256>), dim3(n), dim3(256), 0, st, w.peak_pitch, w.peak_mag, w.peak_cnt,
                     w.n_tframes, w.tf_base, w.tuning_idx, out_tuning);
  CqtArgs ca;
  ca.sig = sig;
  ca.chunk_off = chunk_off;
  ca.oct_off = w.oct_off;
  ca.oct_len = w.oct_len;
  ca.n_frames = w.n_frames;
  ca.tuning_idx = w.tuning_idx;
  ca.ws_oct = w.ws_oct;
  ca.nblk = kCqtBlk;
  ca.tw = ctx.t.tw;
  ca.cqt_lo = ctx.t.cqt_lo;
  ca.cqt_len = ctx.t.cqt_len;
  ca.cqt_off = ctx.t.cqt_off;
  ca.cqt_w = ctx.t.cqt_w;
  ca.cqt_isl = ctx.t.cqt_inv_sqrt_len;
  ca.partial = w.partial;
  const size_t lds = CQ_WAVES * LdsSize<512>::value * sizeof(float2) + kCqtBins * sizeof(float) + 16;
  hipLaunchKernelGGL(cqt_chroma_kernel, dim3(kCqtBlk, n), dim3(CQ_WAVES * 64), lds, st, ca);
  hipLaunchKernelGGL(chroma_finalize_kernel, dim3(n), dim3(64), 0, st, w.partial, kCqtBlk, w.n_frames, n,
                     out_chroma);
  NC_HIP(hipGetLastError());
  return 0;
}

int launch_chroma_lag(const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs, int* lag_out,
                      hipStream_t st) {
  if (n_pairs <= 0) return 0;
  hipLaunchKernelGGL(chroma_lag_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, st, chroma, src_idx, nc_idx,
                     n_pairs, lag_out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

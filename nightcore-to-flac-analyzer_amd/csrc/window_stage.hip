// window_stage.hip — the per-10 s-window tempo features (K1b + K2 + K3 + K4 + K5
// of SURVEY.md §2), in two launches:
//
//   stft_mel_kernel (stft.hip), frame-parallel over every frame of every window:
//     S_db[t][m] = 10 log10(max(1e-10, sum_k mel[m][k] |STFT_2048(x)[k,t]|^2)), frame max,
//     and the f64 energy of the hop slice each frame is centred on;
//   window_tg_kernel, one workgroup per window:
//     energy_db  = 20 log10(max(sqrt(mean(x_f64^2)), 1e-10))           io.py:38-40
//     onset[t]   = mean_m max(0, max(S[t'+1],c) - max(S[t'],c)),  c = max(S) - 80,
//                  t' = t - (1 + n_fft / (2 hop))                      tempo.py:44
//     tg_mean[k] = mean_t ac_t[k] / ac_t[0],  ac_t = autocorr(hann(win) * ramp_pad(onset)[t:t+win])
//                                                                      tempo.py:45/63
//   the autocorrelation evaluated by five sliding f64 sums per lag (nc_slide.h).
// librosa restated in oracle/ncref.py (mel_db, onset_strength, tempogram_mean).
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"
#include "nc_slide.h"

#include "stft_args.h"

namespace nc {

// Tuning knobs (compile-time; tools/wtg_variants.sh sweeps them):
//   NC_WT_SEG   frame segments per window, each an independent set of recurrences
//   NC_WT_PAIR  lags per thread (1, or 2 = k and acw-1-k interleaved)
//   NC_WT_SKIP  diagnosis only: 1 skips the sliding sums, 2 also skips onset + normaliser
#ifndef NC_WT_SEG
#define NC_WT_SEG 1
#endif
#ifndef NC_WT_PAIR
#define NC_WT_PAIR 2
#endif
#ifndef NC_WT_SKIP
#define NC_WT_SKIP 0
#endif
constexpr int WT_SEG = NC_WT_SEG;
constexpr int WT_PAIR = NC_WT_PAIR;
constexpr int WT_WAVES = (WT_PAIR == 2 ? 3 : 6) * WT_SEG;  // ceil(344 / WT_PAIR / 64) waves per segment
constexpr int WT_THREADS = WT_WAVES * 64;

struct WinTgArgs {
  const float* sdb;            // [n_win * T][128]
  const float* frame_max;      // [n_win * T]
  const double* frame_energy;  // [n_win * T]
  const uint8_t* active;       // nullable
  int n_win;
  int T;
  int win_len;
  int pad_onset;
  int acw;
  const double* wsq;  // [acw] Hann(acw)^2
  float* onset_out;   // [n_win][T]
  double* tg_out;     // [n_win][acw]
  double* energy_out; // [n_win]
  unsigned long long* span = nullptr;  // nc_profile execution span (nc_device.h)
};

__global__ __launch_bounds__(WT_THREADS) void window_tg_kernel(WinTgArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ BlockScratch<WT_THREADS> red;
  const int w = blockIdx.x;
  if (a.active && !a.active[w]) return;
  const int T = a.T, acw = a.acw, p = acw / 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* sh_rinv = reinterpret_cast<double*>(smem);          // [T]
  double* sh_x = sh_rinv + T;                                 // [T + acw] ramp-padded onset (f32 values)
  const int64_t g0 = (int64_t)w * T;

  // window max (top_db clamp) and energy, fixed-order reductions
  float m = -INFINITY;
  double e = 0.0;
  for (int i = tid; i < T; i += WT_THREADS) {
    m = fmaxf(m, a.frame_max[g0 + i]);
    e += a.frame_energy[g0 + i];
  }
  const float gmax = (float)block_max((double)m, red);
  const double esum = block_sum(e, red);
  if (tid == 0) a.energy_out[w] = 20.0 * log10(fmax(sqrt(esum / (double)a.win_len), 1e-10));
  const float c = gmax - 80.0f;

  // onset envelope: each wave owns a contiguous run of frames and walks it 8 frames at a
  // time, loading the 9 S_db rows those frames difference (rows shared between neighbours)
  // before using any of them, so 18 row loads per lane are in flight instead of 2
  if (NC_WT_SKIP >= 2) {
    for (int t = tid; t < T; t += WT_THREADS) sh_x[p + t] = 0.0;
  } else {
    constexpr int FB = 8;
    const int per = (T + WT_WAVES - 1) / WT_WAVES;
    const int ta = wave * per, tb = min(T, ta + per);
    // rows of batch t0 + FB are requested before batch t0 is differenced (software pipeline)
    auto load_rows = [&](int t0, float (&ra)[FB + 1], float (&rb)[FB + 1]) {
#pragma unroll
      for (int q = 0; q <= FB; ++q) {
        const int j = t0 + q - a.pad_onset;  // row j feeds frames j + pad (as j) and j + pad - 1 (as j + 1)
        const bool ok = j >= 0 && j < T;
        const float* r = a.sdb + (g0 + (ok ? j : 0)) * 128;
        ra[q] = ok ? r[lane] : 0.0f;
        rb[q] = ok ? r[lane + 64] : 0.0f;
      }
    };
    float ra[FB + 1], rb[FB + 1], na[FB + 1], nb[FB + 1];
    if (ta < tb) load_rows(ta, ra, rb);
    for (int t0 = ta; t0 < tb; t0 += FB) {
      if (t0 + FB < tb) load_rows(t0 + FB, na, nb);
#pragma unroll
      for (int q = 0; q < FB; ++q) {
        const int t = t0 + q;
        if (t >= tb) break;
        float val = 0.0f;
        if (t >= a.pad_onset) {
          const float a0 = fmaxf(ra[q], c), a1 = fmaxf(ra[q + 1], c);
          const float b0 = fmaxf(rb[q], c), b1 = fmaxf(rb[q + 1], c);
          const float part = fmaxf(0.0f, a1 - a0) + fmaxf(0.0f, b1 - b0);
          val = wave_sum(part) * (1.0f / 128.0f);
        }
        if (lane == 0) {
          sh_x[p + t] = val;
          a.onset_out[g0 + t] = val;
        }
      }
#pragma unroll
      for (int q = 0; q <= FB; ++q) {
        ra[q] = na[q];
        rb[q] = nb[q];
      }
    }
  }
  __syncthreads();
  {  // linear_ramp padding to 0 at both ends (numpy.pad, f64 ramp rounded to f32)
    const double st0 = sh_x[p] / (double)p, stl = sh_x[p + T - 1] / (double)p;
    for (int i = tid; i < p; i += WT_THREADS) {
      sh_x[i] = (double)(float)((double)i * st0);
      sh_x[p + T + i] = (double)(float)((double)(p - 1 - i) * stl);
    }
  }
  __syncthreads();
  // per-frame normaliser 1 / ac_t[0] = 1 / sum_j hann[j]^2 x[t+j]^2: Hann^2 staged in LDS,
  // four interleaved partial sums per frame (independent FMA chains), joined in a fixed order
  double* sh_wsq = sh_x + (T + acw) + WT_SEG * acw;
  for (int j = tid; j < acw; j += WT_THREADS) sh_wsq[j] = a.wsq[j];
  __syncthreads();
  for (int t = tid; t < T; t += WT_THREADS) {
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    const int n = NC_WT_SKIP >= 2 ? 0 : acw;
    int j = 0;
    for (; j + 4 <= n; j += 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double v = sh_x[t + j + q];
        s4[q] = fma(sh_wsq[j + q], v * v, s4[q]);
      }
    }
    for (; j < n; ++j) {
      const double v = sh_x[t + j];
      s4[0] = fma(sh_wsq[j], v * v, s4[0]);
    }
    sh_rinv[t] = tg_rinv((s4[0] + s4[1]) + (s4[2] + s4[3]));
  }
  __syncthreads();
  auto xf = [&](int i) { return sh_x[i]; };
  auto rf = [&](int t) { return sh_rinv[t]; };
  // lags k and acw-1-k per thread: two independent f64 recurrences (latency hiding), and
  // their start-up sums (acw - k and k + 1 terms) add up to the same work on every thread;
  // the frames are split into WT_SEG segments, each started by its own direct sums, and
  // the segment partials are added in segment order
  double* part = sh_x + (T + acw);  // [WT_SEG][acw]
  const int seg = tid / (WT_THREADS / WT_SEG), st = tid % (WT_THREADS / WT_SEG);
  const int ta = T * seg / WT_SEG, tb = T * (seg + 1) / WT_SEG;
  if (NC_WT_SKIP == 0) {
    if (WT_PAIR == 2) {
      for (int i = st; i < (acw + 1) / 2; i += WT_THREADS / WT_SEG) {
        const int ka = i, kb = acw - 1 - i;
        double sa, sb;
        slide_lag_sum2(xf, rf, acw, ka, kb, ta, tb, sa, sb);
        part[seg * acw + ka] = sa;
        if (kb != ka) part[seg * acw + kb] = sb;
      }
    } else {
      for (int k = st; k < acw; k += WT_THREADS / WT_SEG) part[seg * acw + k] = slide_lag_sum(xf, rf, acw, k, ta, tb);
    }
  } else {
    for (int k = st; k < acw; k += WT_THREADS / WT_SEG) part[seg * acw + k] = 0.0;
  }
  __syncthreads();
  for (int k = tid; k < acw; k += WT_THREADS) {
    double acc = part[k];
#pragma unroll
    for (int q = 1; q < WT_SEG; ++q) acc += part[q * acw + k];
    a.tg_out[(size_t)w * acw + k] = acc / (double)T;
  }
}

static inline size_t a256(size_t n) { return (n + 255) & ~(size_t)255; }

size_t window_stage_ws_bytes(const Context&, int n_win, int T) {
  const size_t F = (size_t)n_win * T;
  return a256(F * 128 * sizeof(float)) + a256(F * sizeof(float)) + a256(F * sizeof(double));
}

int launch_window_stage(Context& ctx, const float* sig, const int64_t* win_off, const uint8_t* active,
                        int n_win, int win_len, int hop, float* onset_out, double* tg_out,
                        double* energy_out, const int* win_chunk, const int64_t* chunk_tf_base, int tp_frames,
                        float* peak_pitch, float* peak_mag, int* chunk_npk, void* stft_done,
                        void* ws, size_t ws_bytes, hipStream_t st) {
  if (n_win <= 0) return 0;
  if (hop != 512) {
    set_error("window stage: only hop_length=512 is supported (tempo.py:24)");
    return -2;
  }
  const int T = 1 + win_len / hop;
  const int acw = ctx.t.ac512;
  if (ws_bytes < window_stage_ws_bytes(ctx, n_win, T)) {
    set_error("window stage: workspace too small");
    return -3;
  }
  const size_t F = (size_t)n_win * T;
  char* q = static_cast<char*>(ws);
  float* sdb = reinterpret_cast<float*>(q);
  q += a256(F * 128 * sizeof(float));
  float* fmax_ = reinterpret_cast<float*>(q);
  q += a256(F * sizeof(float));
  double* fen = reinterpret_cast<double*>(q);

  StftMelArgs s{};
  s.sig = sig;
  s.seq_off = win_off;
  s.seq_len = nullptr;
  s.frame_base = nullptr;
  s.uniform_len = win_len;
  s.uniform_T = T;
  s.n_seq = n_win;
  s.total_frames = (int64_t)F;
  s.active = active;
  s.hop = hop;
  s.sdb = sdb;
  s.frame_max = fmax_;
  s.frame_energy = fen;
  if (win_chunk) {
    // a shared frame must see no right-edge padding of the window: t hop + n_fft / 2 <= win_len
    if (!chunk_tf_base || !peak_pitch || !peak_mag || !chunk_npk || tp_frames < 0 || tp_frames > T ||
        (tp_frames > 0 && (int64_t)(tp_frames - 1) * hop + kNFFT / 2 > win_len)) {
      set_error("window stage: shared tuning frames need chunk bases, peak lists and frames inside the window");
      return -2;
    }
    s.win_chunk = win_chunk;
    s.chunk_tf_base = chunk_tf_base;
    s.tp_frames = tp_frames;
    s.peak_pitch = peak_pitch;
    s.peak_mag = peak_mag;
    s.chunk_npk = chunk_npk;
  }
  int rc = launch_stft_mel(ctx, s, st);
  if (rc) return rc;
  // the shared tuning peaks are complete here: a chroma chain on another stream may go on
  if (stft_done) NC_HIP(hipEventRecord(static_cast<hipEvent_t>(stft_done), st));

  WinTgArgs a;
  a.sdb = sdb;
  a.frame_max = fmax_;
  a.frame_energy = fen;
  a.active = active;
  a.n_win = n_win;
  a.T = T;
  a.win_len = win_len;
  a.pad_onset = 1 + kNFFT / (2 * hop);
  a.acw = acw;
  a.wsq = ctx.t.wsq512;
  a.onset_out = onset_out;
  a.tg_out = tg_out;
  a.energy_out = energy_out;
  const size_t lds = (size_t)T * sizeof(double) + (size_t)(T + acw + WT_SEG * acw + acw) * sizeof(double);
  if (lds > 160 * 1024) {
    set_error("window stage: window too long for LDS (window_sec above ~225 s at hop 512)");
    return -2;
  }
  {
    KTimer kt_(ctx, "window_tg", st);
    a.span = kt_.span();
    hipLaunchKernelGGL(window_tg_kernel, dim3(n_win), dim3(WT_THREADS), lds, st, a);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

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

constexpr int WT_WAVES = 6;
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
};

__global__ __launch_bounds__(WT_THREADS) void window_tg_kernel(WinTgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ BlockScratch<WT_THREADS> red;
  const int w = blockIdx.x;
  if (a.active && !a.active[w]) return;
  const int T = a.T, acw = a.acw, p = acw / 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* sh_rinv = reinterpret_cast<double*>(smem);          // [T]
  float* sh_x = reinterpret_cast<float*>(sh_rinv + T);        // [T + acw] ramp-padded onset
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

  // onset envelope: one wave per frame, lanes over bands
  for (int t = wave; t < T; t += WT_WAVES) {
    float val = 0.0f;
    if (t >= a.pad_onset) {
      const float* r0 = a.sdb + (g0 + t - a.pad_onset) * 128;
      const float* r1 = r0 + 128;
      const float a0 = fmaxf(r0[lane], c), a1 = fmaxf(r1[lane], c);
      const float b0 = fmaxf(r0[lane + 64], c), b1 = fmaxf(r1[lane + 64], c);
      const float part = fmaxf(0.0f, a1 - a0) + fmaxf(0.0f, b1 - b0);
      val = wave_sum(part) * (1.0f / 128.0f);
    }
    if (lane == 0) {
      sh_x[p + t] = val;
      a.onset_out[g0 + t] = val;
    }
  }
  __syncthreads();
  {  // linear_ramp padding to 0 at both ends (numpy.pad, f64 ramp rounded to f32)
    const double st0 = (double)sh_x[p] / (double)p, stl = (double)sh_x[p + T - 1] / (double)p;
    for (int i = tid; i < p; i += WT_THREADS) {
      sh_x[i] = (float)((double)i * st0);
      sh_x[p + T + i] = (float)((double)(p - 1 - i) * stl);
    }
  }
  __syncthreads();
  // per-frame normaliser 1 / ac_t[0]
  for (int t = tid; t < T; t += WT_THREADS) {
    double s = 0.0;
    for (int j = 0; j < acw; ++j) {
      const double v = (double)sh_x[t + j];
      s = fma(a.wsq[j], v * v, s);
    }
    sh_rinv[t] = tg_rinv(s);
  }
  __syncthreads();
  auto xf = [&](int i) { return sh_x[i]; };
  auto rf = [&](int t) { return sh_rinv[t]; };
  for (int k = tid; k < acw; k += WT_THREADS) {
    const double acc = slide_lag_sum(xf, rf, acw, k, 0, T);
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
                        double* energy_out, void* ws, size_t ws_bytes, hipStream_t st) {
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
  int rc = launch_stft_mel(ctx, s, st);
  if (rc) return rc;

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
  const size_t lds = (size_t)T * sizeof(double) + (size_t)(T + acw) * sizeof(float);
  if (lds > 64 * 1024) {
    set_error("window stage: window too long for LDS");
    return -2;
  }
  {
    KTimer kt_(ctx, "window_tg", st);
    hipLaunchKernelGGL(window_tg_kernel, dim3(n_win), dim3(WT_THREADS), lds, st, a);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

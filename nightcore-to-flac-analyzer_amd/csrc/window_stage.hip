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
//   the lag sums evaluated as six correlations of prefix-sum sequences (nc_tgcorr.h).
// librosa restated in oracle/ncref.py (mel_db, onset_strength, tempogram_mean).
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"
#include "nc_slide.h"
#include "nc_tgcorr.h"

#include "stft_args.h"

namespace nc {

// The tempogram sum is evaluated as six lag correlations (nc_tgcorr.h): per window,
//   T tg_mean[k] = sum_{i<3} phi_i(k) (Hank_i(k) - Toep_i(k)),  phi = (1, cos theta k, sin theta k),
//   Hank_i(k) = sum_u a_i[u] x[u + k],  Toep_i(k) = sum_u b_i[u] x[u - k],
// with a_i / b_i built from prefix sums of the frame normalisers (derivation in nc_tgcorr.h).
constexpr int WT_THREADS = 512;  // 8 waves; ~78 KB LDS -> two windows per CU
constexpr size_t kWinTgLdsCap = 160 * 1024 - 1024;  // dynamic LDS; the rest holds BlockScratch

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

// LDS carve-up of one window (doubles), shared by the kernel and its launcher.
struct WinTgLds {
  int T, acw, U, xoff, xlen, seq, scr, scr_len, total;
  __host__ __device__ WinTgLds(int T_, int acw_) : T(T_), acw(acw_) {
    U = tgc_extent(T, acw);
    xoff = tgc_pad(acw);                          // x[i] at xoff + i; zeros outside [0, T + 2 (acw / 2))
    xlen = U + 2 * xoff;
    seq = xlen;                                   // [6][U] correlation sequences
    const int pre = T + acw + 2 * acw + 5 * (T + 1);  // rinv, Hann^2, (cos, sin) table, prefix sums
    const int post = tgc_segments(acw, WT_THREADS) * tgc_blocks(acw) * TGC_LB;  // per-segment partials
    scr = seq + 6 * U;
    scr_len = pre > post ? pre : post;
    total = scr + scr_len;
  }
};

// Window max (top_db clamp) and energy, then the ramp-padded onset envelope into
// x[0, T + 2 (acw / 2)).  Each wave owns a contiguous run of frames and walks it 8 frames
// at a time, loading the 9 S_db rows those frames difference (rows shared between
// neighbours) before using any of them, so 9 row loads per lane are in flight instead of 1.
template <int NT>
__device__ __forceinline__ void wtg_onset(const WinTgArgs& a, int w, double* sh_x, BlockScratch<NT>& red) {
  const int T = a.T, p = a.acw / 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t g0 = (int64_t)w * T;
  float m = -INFINITY;
  double e = 0.0;
  for (int i = tid; i < T; i += NT) {
    m = fmaxf(m, a.frame_max[g0 + i]);
    if (a.frame_energy) e += a.frame_energy[g0 + i];
  }
  const float gmax = (float)block_max((double)m, red);
  if (a.frame_energy) {  // else nc_window_energy_blocks gives the energy from the trim's block sums
    const double esum = block_sum(e, red);
    if (tid == 0) a.energy_out[w] = 20.0 * log10(fmax(sqrt(esum / (double)a.win_len), 1e-10));
  }
  const float c = gmax - 80.0f;

  constexpr int FB = 8, NW = NT / 64;
  const int per = (T + NW - 1) / NW;
  const int ta = wave * per, tb = min(T, ta + per);
  // lane l holds bands 2l, 2l+1 of a row (one 8-byte load per row); rows of batch t0 + FB
  // are requested before batch t0 is differenced (software pipeline)
  auto load_rows = [&](int t0, float2 (&ra)[FB + 1]) {
#pragma unroll
    for (int q = 0; q <= FB; ++q) {
      const int j = t0 + q - a.pad_onset;  // row j feeds frames j + pad (as j) and j + pad - 1 (as j + 1)
      const bool ok = j >= 0 && j < T;
      const float2* r = reinterpret_cast<const float2*>(a.sdb + (g0 + (ok ? j : 0)) * 128);
      ra[q] = ok ? r[lane] : make_float2(0.0f, 0.0f);
    }
  };
  float2 ra[FB + 1], na[FB + 1];
  if (ta < tb) load_rows(ta, ra);
  for (int t0 = ta; t0 < tb; t0 += FB) {
    if (t0 + FB < tb) load_rows(t0 + FB, na);
    float part[FB];
#pragma unroll
    for (int q = 0; q < FB; ++q) {
      const float a0 = fmaxf(ra[q].x, c), a1 = fmaxf(ra[q + 1].x, c);
      const float b0 = fmaxf(ra[q].y, c), b1 = fmaxf(ra[q + 1].y, c);
      part[q] = fmaxf(0.0f, a1 - a0) + fmaxf(0.0f, b1 - b0);
    }
    // transposed reduction of the FB = 8 frame partials: lane bits 5, 4, 3 halve the
    // frame set (4 + 2 + 1 exchanges), bits 2..0 finish one frame per lane (3): frame f's
    // band sum ends in lane 8 f
    {
      const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8;
      float p4[4], p2[2], p1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float keep = h5 ? part[q + 4] : part[q], give = h5 ? part[q] : part[q + 4];
        p4[q] = keep + __shfl_xor(give, 32, 64);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float keep = h4 ? p4[q + 2] : p4[q], give = h4 ? p4[q] : p4[q + 2];
        p2[q] = keep + __shfl_xor(give, 16, 64);
      }
      {
        const float keep = h3 ? p2[1] : p2[0], give = h3 ? p2[0] : p2[1];
        p1 = keep + __shfl_xor(give, 8, 64);
      }
      p1 += __shfl_xor(p1, 4, 64);
      p1 += __shfl_xor(p1, 2, 64);
      p1 += __shfl_xor(p1, 1, 64);
      const int f = lane >> 3, t = t0 + f;
      if ((lane & 7) == 0 && t < tb) {
        const float val = t >= a.pad_onset ? p1 * (1.0f / 128.0f) : 0.0f;
        sh_x[p + t] = val;
        a.onset_out[g0 + t] = val;
      }
    }
#pragma unroll
    for (int q = 0; q <= FB; ++q) ra[q] = na[q];
  }
  __syncthreads();
  {  // linear_ramp padding to 0 at both ends (numpy.pad, f64 ramp rounded to f32)
    const double st0 = sh_x[p] / (double)p, stl = sh_x[p + T - 1] / (double)p;
    for (int i = tid; i < p; i += NT) {
      sh_x[i] = (double)(float)((double)i * st0);
      sh_x[p + T + i] = (double)(float)((double)(p - 1 - i) * stl);
    }
  }
  __syncthreads();
}

// Per-frame normaliser 1 / ac_t[0] = 1 / sum_j hann[j]^2 x[t+j]^2 (Hann^2 in LDS), four
// interleaved partial sums per frame (independent FMA chains) joined in a fixed order.
template <int NT>
__device__ __forceinline__ void wtg_rinv(const double* sh_x, const double* sh_wsq, int T, int acw, double* sh_rinv) {
  for (int t = threadIdx.x; t < T; t += NT) {
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    int j = 0;
    for (; j + 4 <= acw; j += 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double v = sh_x[t + j + q];
        s4[q] = fma(sh_wsq[j + q], v * v, s4[q]);
      }
    }
    for (; j < acw; ++j) {
      const double v = sh_x[t + j];
      s4[0] = fma(sh_wsq[j], v * v, s4[0]);
    }
    sh_rinv[t] = tg_rinv((s4[0] + s4[1]) + (s4[2] + s4[3]));
  }
}

// The same normalisers register-blocked: 5 consecutive frames x 1/5 of the taps per
// thread over y = x^2, the five tap-segment partials added in segment order.
// y [T + acw] and part [5][T] are LDS scratch.
template <int NT>
__device__ __forceinline__ void wtg_rinv_blocked(const double* sh_x, const double* sh_wsq, int T, int acw, double* y,
                                                 double* part, double* sh_rinv) {
  constexpr int RB = 5, JS = 5;
  const int tid = threadIdx.x;
  for (int i = tid; i < T + acw; i += NT) y[i] = sh_x[i] * sh_x[i];
  __syncthreads();
  const int nb = (T + RB - 1) / RB;
  for (int task = tid; task < nb * JS; task += NT) {
    const int b = task % nb, js = task / nb, t0 = b * RB;
    const int ja = acw * js / JS, jb = acw * (js + 1) / JS;
    double acc[RB], yw[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      acc[q] = 0.0;
      yw[q] = q < RB - 1 ? y[min(t0 + ja + q, T + acw - 1)] : 0.0;
    }
#pragma unroll 1
    for (int j = ja; j < jb; ++j) {
      yw[RB - 1] = y[min(t0 + j + RB - 1, T + acw - 1)];
      const double wj = sh_wsq[j];
#pragma unroll
      for (int q = 0; q < RB; ++q) acc[q] = fma(wj, yw[q], acc[q]);
#pragma unroll
      for (int q = 0; q < RB - 1; ++q) yw[q] = yw[q + 1];
    }
#pragma unroll
    for (int q = 0; q < RB; ++q)
      if (t0 + q < T) part[js * T + t0 + q] = acc[q];
  }
  __syncthreads();
  for (int t = tid; t < T; t += NT) {
    double s = part[t];
#pragma unroll
    for (int q = 1; q < JS; ++q) s += part[q * T + t];
    sh_rinv[t] = tg_rinv(s);
  }
}

__global__ __launch_bounds__(WT_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void window_tg_kernel(WinTgArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ BlockScratch<WT_THREADS> red;
  const int w = blockIdx.x;
  if (a.active && !a.active[w]) return;
  const int T = a.T, acw = a.acw, p = acw / 2, tid = threadIdx.x;
  const WinTgLds L(T, acw);
  double* lds = reinterpret_cast<double*>(smem);
  double* sh_x = lds + L.xoff;    // ramp-padded onset (f32 values), zeros either side
  double* seq = lds + L.seq;      // [6][U]
  double* sh_rinv = lds + L.scr;  // [T]
  double* sh_wsq = sh_rinv + T;   // [acw]
  double* sh_cs = sh_wsq + acw;   // [acw][2] (cos, sin)(theta j)
  double* sh_q = sh_cs + 2 * acw; // [5][T + 1] prefix sums

  for (int i = tid; i < L.xoff; i += WT_THREADS) lds[i] = 0.0;
  for (int i = T + 2 * p + tid; i < L.xlen - L.xoff; i += WT_THREADS) sh_x[i] = 0.0;
  for (int j = tid; j < acw; j += WT_THREADS) {
    sh_wsq[j] = a.wsq[j];
    double s, cc;
    sincospi(2.0 * (double)j / (double)acw, &s, &cc);
    sh_cs[2 * j] = cc;
    sh_cs[2 * j + 1] = s;
  }
  wtg_onset<WT_THREADS>(a, w, sh_x, red);
  wtg_rinv_blocked<WT_THREADS>(sh_x, sh_wsq, T, acw, seq, sh_q, sh_rinv);
  __syncthreads();
  tgc_prefix(sh_rinv, sh_cs, T, acw, sh_q, tid, WT_THREADS);
  __syncthreads();
  tgc_sequences(sh_x, sh_q, sh_cs, T, acw, L.U, seq, tid, WT_THREADS);
  __syncthreads();
  double* part = lds + L.scr;  // [segments][blocks * LB], over the normaliser scratch
  tgc_correlate(sh_x, seq, acw, L.U, part, tid, WT_THREADS);
  __syncthreads();
  const int nseg = tgc_segments(acw, WT_THREADS), stride = tgc_blocks(acw) * TGC_LB;
  for (int k = tid; k < acw; k += WT_THREADS) {
    double acc = part[k];
    for (int q = 1; q < nseg; ++q) acc += part[q * stride + k];
    a.tg_out[(size_t)w * acw + k] = acc / (double)T;
  }
}

// Windows whose correlation sequences do not fit in LDS (window_sec above ~29 s): the
// sliding sums of nc_slide.h, lags k and acw-1-k per thread (equal start-up work).
constexpr int WS_THREADS = 192;
__host__ __device__ inline size_t wtg_slide_lds_doubles(int T, int acw) { return (size_t)T + (T + acw) + 2 * (size_t)acw; }

__global__ __launch_bounds__(WS_THREADS) void window_tg_slide_kernel(WinTgArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ BlockScratch<WS_THREADS> red;
  const int w = blockIdx.x;
  if (a.active && !a.active[w]) return;
  const int T = a.T, acw = a.acw, tid = threadIdx.x;
  double* sh_rinv = reinterpret_cast<double*>(smem);  // [T]
  double* sh_x = sh_rinv + T;                         // [T + acw]
  double* part = sh_x + (T + acw);                    // [acw]
  double* sh_wsq = part + acw;                        // [acw]
  for (int j = tid; j < acw; j += WS_THREADS) sh_wsq[j] = a.wsq[j];
  wtg_onset<WS_THREADS>(a, w, sh_x, red);
  wtg_rinv<WS_THREADS>(sh_x, sh_wsq, T, acw, sh_rinv);
  __syncthreads();
  auto xf = [&](int i) { return sh_x[i]; };
  auto rf = [&](int t) { return sh_rinv[t]; };
  for (int i = tid; i < (acw + 1) / 2; i += WS_THREADS) {
    const int ka = i, kb = acw - 1 - i;
    double sa, sb;
    slide_lag_sum2(xf, rf, acw, ka, kb, 0, T, sa, sb);
    part[ka] = sa;
    if (kb != ka) part[kb] = sb;
  }
  __syncthreads();
  for (int k = tid; k < acw; k += WS_THREADS) a.tg_out[(size_t)w * acw + k] = part[k] / (double)T;
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
  s.frame_energy = energy_out ? fen : nullptr;
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
  a.frame_energy = energy_out ? fen : nullptr;
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
  // the correlation kernel while its sequences fit in LDS (~104 B / frame: two windows
  // per CU at the default 10 s, one up to ~29 s), else the sliding sums (~16 B / frame:
  // up to ~225 s)
  const size_t lds_corr = (size_t)WinTgLds(T, acw).total * sizeof(double);
  const size_t lds_slide = wtg_slide_lds_doubles(T, acw) * sizeof(double);
  const bool corr = lds_corr <= kWinTgLdsCap;
  if (!corr && lds_slide > kWinTgLdsCap) {
    set_error("window stage: window too long for LDS (window_sec above ~225 s at hop 512)");
    return -2;
  }
  {
    KTimer kt_(ctx, "window_tg", st);
    a.span = kt_.span();
    if (corr)
      for (int rep = 0; rep < NC_PROBE_REPS(2); ++rep)
        hipLaunchKernelGGL(window_tg_kernel, dim3(n_win), dim3(WT_THREADS), lds_corr, st, a);
    else
      hipLaunchKernelGGL(window_tg_slide_kernel, dim3(n_win), dim3(WS_THREADS), lds_slide, st, a);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

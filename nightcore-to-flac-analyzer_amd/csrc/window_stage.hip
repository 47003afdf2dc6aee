// window_stage.hip — the per-10 s-window hot path, fused in one persistent
// workgroup per window (K1b + K2 + K3 + K4 + K5 of SURVEY.md §2):
//
//   energy_db   = 20 log10(max(sqrt(mean(x_f64^2)), 1e-10))          io.py:38-40
//   S_db[t][m]  = 10 log10(max(1e-10, sum_k mel[m][k] |STFT_2048(x)[k,t]|^2))
//   onset[t]    = mean_m max(0, max(S[t'+1],c) - max(S[t'],c)),  c = max(S) - 80,
//                 t' = t - (1 + n_fft / (2 hop))                     tempo.py:44
//   tg_mean[k]  = mean_t ac_t[k] / max|ac_t|,  ac_t = autocorr(hann(win) * ramp_pad(onset)[t:t+win])
//                                                                    tempo.py:45/63
// librosa restated in oracle/ncref.py (onset_strength, tempogram_mean).
//
// MI355X layout: one workgroup (4 waves) per window, persistent over windows;
// each wave owns whole STFT frames (1024-point complex FFT = 2048 real, Stockham
// radix 16.16.4 through an 8.7 KB LDS slot); S_db for the window goes to a
// per-workgroup global scratch slot (220 KB, L2 / Infinity-Cache resident since
// the slot is reused window after window) because the top_db clamp needs the
// window-global max before any difference can be taken.  The tempogram runs
// from LDS (onset envelope, ramp-padded) with 512-point complex FFT pairs.
#include "nc_device.h"
#include "nc_engine.h"
#include <algorithm>

namespace nc {

constexpr int WS_WAVES = 4;
constexpr int WS_THREADS = WS_WAVES * 64;

struct WinArgs {
  const float* sig;
  const int64_t* win_off;
  const uint8_t* active;  // nullable: skip windows with active[w] == 0
  int n_win;
  int win_len;
  int hop;
  int T;
  int pad_onset;
  int acw;
  float* sdb_ws;      // [gridDim.x][T][128]
  float* onset_out;   // [n_win][T]
  double* tg_out;     // [n_win][acw]
  double* energy_out; // [n_win]
  const float2* tw;
  const float* hann2048;
  const float* wac;
  const int* mel_lo;
  const int* mel_len;
  const int* mel_off;
  const float* mel_w;
};

__host__ __device__ __forceinline__ int align4(int n) { return (n + 3) & ~3; }

__global__ __launch_bounds__(WS_THREADS) void window_stage_kernel(WinArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float2* fft_all = reinterpret_cast<float2*>(smem);
  float2* fftbuf = fft_all + wave * LdsSize<1024>::value;
  float* sh_region = reinterpret_cast<float*>(fft_all + WS_WAVES * LdsSize<1024>::value);
  float* sh_hann = sh_region;                         // 2048 floats (phase 1)
  float* sh_opad = sh_region;                         // T + acw floats (phase 4, reuses hann)
  float* sh_wac = sh_region + align4(a.T + a.acw);    // acw floats (phase 4)
  float* sh_onset = sh_region + max(2048, align4(a.T + a.acw) + align4(a.acw));
  __shared__ float sh_redf[WS_WAVES];
  __shared__ double sh_redd[WS_WAVES];

  const int T = a.T, acw = a.acw;
  float* sdb = a.sdb_ws + (size_t)blockIdx.x * T * 128;

  for (int w = blockIdx.x; w < a.n_win; w += gridDim.x) {
    if (a.active && !a.active[w]) continue;
    const float* x = a.sig + a.win_off[w];
    const int L = a.win_len;

    // ---------------------------------------------------------------- phase 0: energy (f64)
    for (int i = threadIdx.x; i < 2048; i += WS_THREADS) sh_hann[i] = a.hann2048[i];
    double e = 0.0;
    for (int i = threadIdx.x; i < L; i += WS_THREADS) {
      const double v = (double)x[i];
      e = fma(v, v, e);
    }
    e = wave_sum(e);
    if (lane == 0) sh_redd[wave] = e;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int i = 0; i < WS_WAVES; ++i) s += sh_redd[i];
      const double rms = sqrt(s / (double)L);
      a.energy_out[w] = 20.0 * log10(fmax(rms, 1e-10));
    }

    // ---------------------------------------------------------------- phase 1: STFT -> mel dB
    float lmax = -INFINITY;
    for (int t = wave; t < T; t += WS_WAVES) {
      const int s0 = t * a.hop - 1024;
      FftIn<1024> in;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = lane + 64 * r;
        const int i0 = s0 + 2 * n;
        const float x0 = (i0 >= 0 && i0 < L) ? x[i0] : 0.0f;
        const float x1 = (i0 + 1 >= 0 && i0 + 1 < L) ? x[i0 + 1] : 0.0f;
        in[0][r] = make_float2(x0 * sh_hann[2 * n], x1 * sh_hann[2 * n + 1]);
      }
      wave_fft<1024>(in, fftbuf, a.tw, lane);
      float p1[9], p2[9];
#pragma unroll
      for (int m = 0; m < 9; ++m) {
        const int k = lane + 64 * m;
        if (k <= 512) {
          float2 X, XN;
          rfft_split(fftbuf, a.tw, 1024, k, X, XN);
          p1[m] = fmaf(X.x, X.x, X.y * X.y);
          p2[m] = fmaf(XN.x, XN.x, XN.y * XN.y);
        }
      }
      float* pw = reinterpret_cast<float*>(fftbuf);
#pragma unroll
      for (int m = 0; m < 9; ++m) {
        const int k = lane + 64 * m;
        if (k <= 512) {
          pw[k] = p1[m];
          pw[1024 - k] = p2[m];
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int b = h == 0 ? lane : 127 - lane;
        const int lo = a.mel_lo[b], len = a.mel_len[b], off = a.mel_off[b];
        float acc = 0.0f;
        for (int j = 0; j < len; ++j) acc = fmaf(a.mel_w[off + j], pw[lo + j], acc);
        const float db = 10.0f * log10f(fmaxf(1e-10f, acc));
        sdb[t * 128 + b] = db;
        lmax = fmaxf(lmax, db);
      }
    }
    lmax = wave_max(lmax);
    if (lane == 0) sh_redf[wave] = lmax;
    __syncthreads();
    float gmax = sh_redf[0];
#pragma unroll
    for (int i = 1; i < WS_WAVES; ++i) gmax = fmaxf(gmax, sh_redf[i]);
    const float c = gmax - 80.0f;

    // ---------------------------------------------------------------- phase 3: onset envelope
    for (int t = wave; t < T; t += WS_WAVES) {
      float val = 0.0f;
      if (t >= a.pad_onset) {
        const int j = t - a.pad_onset;
        const float a0 = fmaxf(sdb[j * 128 + lane], c), a1 = fmaxf(sdb[(j + 1) * 128 + lane], c);
        const float b0 = fmaxf(sdb[j * 128 + lane + 64], c), b1 = fmaxf(sdb[(j + 1) * 128 + lane + 64], c);
        const float part = fmaxf(0.0f, a1 - a0) + fmaxf(0.0f, b1 - b0);
        val = wave_sum(part) * (1.0f / 128.0f);
      }
      if (lane == 0) {
        sh_onset[t] = val;
        a.onset_out[(size_t)w * T + t] = val;
      }
    }
    __syncthreads();

    // ---------------------------------------------------------------- phase 4: tempogram mean
    const int p = acw / 2;
    {
      const double x0 = (double)sh_onset[0], xl = (double)sh_onset[T - 1];
      const double st0 = x0 / (double)p, stl = xl / (double)p;
      for (int i = threadIdx.x; i < T + 2 * p; i += WS_THREADS) {
        float v;
        if (i < p) v = (float)((double)i * st0);
        else if (i < p + T) v = sh_onset[i - p];
        else v = (float)((double)(p - 1 - (i - p - T)) * stl);
        sh_opad[i] = v;
      }
      for (int i = threadIdx.x; i < acw; i += WS_THREADS) sh_wac[i] = a.wac[i];
    }
    __syncthreads();

    constexpr int NQ = 4;  // lags 2n, 2n+1 for n = lane + 64 q  (acw <= 512)
    double acc[NQ][2];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q][0] = acc[q][1] = 0.0;

    for (int t = wave; t < T; t += WS_WAVES) {
      FftIn<512> in;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int j0 = 2 * (lane + 64 * r);
        const float v0 = j0 < acw ? sh_opad[t + j0] * sh_wac[j0] : 0.0f;
        const float v1 = j0 + 1 < acw ? sh_opad[t + j0 + 1] * sh_wac[j0 + 1] : 0.0f;
        in[0][r] = make_float2(v0, v1);
      }
      wave_fft<512>(in, fftbuf, a.tw, lane);
      float pk[5], pn[5];
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const int k = lane + 64 * m;
        if (k <= 256) {
          float2 X, XN;
          rfft_split(fftbuf, a.tw, 512, k, X, XN);
          pk[m] = fmaf(X.x, X.x, X.y * X.y);
          pn[m] = fmaf(XN.x, XN.x, XN.y * XN.y);
        }
      }
      float* pw = reinterpret_cast<float*>(fftbuf);
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const int k = lane + 64 * m;
        if (k <= 256) {
          pw[k] = pk[m];
          pw[512 - k] = pn[m];
        }
      }
      // conj(Z'[n]), Z'[n] = E + i O e^{+2 pi i n/1024}
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int n = lane + 64 * r;
        const float Pa = pw[n], Pb = pw[512 - n];
        const float E = 0.5f * (Pa + Pb), Od = 0.5f * (Pa - Pb);
        const float2 wv = a.tw[(8 * n) & 8191];  // exp(-2 pi i n/1024) = (cos, -sin)
        const float cs = wv.x, sn = -wv.y;
        in[0][r] = make_float2(E - Od * sn, -(Od * cs));
      }
      wave_fft<512>(in, fftbuf, a.tw, lane);
      float av[NQ][2];
      float mx = 0.0f;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int n = lane + 64 * q;
        av[q][0] = av[q][1] = 0.0f;
        if (2 * n < acw) {
          const float2 y = fftbuf[lpad(n)];
          av[q][0] = y.x;
          av[q][1] = (2 * n + 1 < acw) ? -y.y : 0.0f;
        }
        mx = fmaxf(mx, fmaxf(fabsf(av[q][0]), fabsf(av[q][1])));
      }
      mx = wave_max(mx);
      const double inv = (mx < 1.17549435e-38f) ? 1.0 : 1.0 / (double)mx;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        acc[q][0] += (double)av[q][0] * inv;
        acc[q][1] += (double)av[q][1] * inv;
      }
    }
    __syncthreads();  // all FFT slots free: reuse them for the cross-wave sum
    double* red = reinterpret_cast<double*>(fft_all);  // [WS_WAVES][acw]
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int n = lane + 64 * q;
      if (2 * n < acw) red[wave * acw + 2 * n] = acc[q][0];
      if (2 * n + 1 < acw) red[wave * acw + 2 * n + 1] = acc[q][1];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < acw; k += WS_THREADS) {
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < WS_WAVES; ++i) s += red[i * acw + k];
      a.tg_out[(size_t)w * acw + k] = s / (double)T;
    }
    __syncthreads();
  }
}

size_t window_stage_lds_bytes(int T, int acw) {
  const size_t fft = (size_t)WS_WAVES * LdsSize<1024>::value * sizeof(float2);
  const size_t region = (size_t)std::max(2048, align4(T + acw) + align4(acw)) + (size_t)align4(T);
  return fft + region * sizeof(float);
}

int window_stage_grid(const Context& ctx, int n_win) {
  return std::max(1, std::min(n_win, 3 * ctx.num_cu));
}

size_t window_stage_ws_bytes(const Context& ctx, int n_win, int T) {
  return (size_t)window_stage_grid(ctx, n_win) * T * 128 * sizeof(float);
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
  if (acw > 512 || 2 * acw - 1 > 1024) {
    set_error("window stage: tempogram window too long");
    return -2;
  }
  if (ws_bytes < window_stage_ws_bytes(ctx, n_win, T)) {
    set_error("window stage: workspace too small");
    return -3;
  }
  WinArgs a;
  a.sig = sig;
  a.win_off = win_off;
  a.active = active;
  a.n_win = n_win;
  a.win_len = win_len;
  a.hop = hop;
  a.T = T;
  a.pad_onset = 1 + kNFFT / (2 * hop);
  a.acw = acw;
  a.sdb_ws = static_cast<float*>(ws);
  a.onset_out = onset_out;
  a.tg_out = tg_out;
  a.energy_out = energy_out;
  a.tw = ctx.t.tw;
  a.hann2048 = ctx.t.hann2048;
  a.wac = ctx.t.hann_ac512;
  a.mel_lo = ctx.t.mel_lo;
  a.mel_len = ctx.t.mel_len;
  a.mel_off = ctx.t.mel_off;
  a.mel_w = ctx.t.mel_w;
  const size_t lds = window_stage_lds_bytes(T, acw);
  if (lds > 160 * 1024) {
    set_error("window stage: window too long for LDS");
    return -2;
  }
  const int grid = window_stage_grid(ctx, n_win);
  hipLaunchKernelGGL(window_stage_kernel, dim3(grid), dim3(WS_THREADS), lds, st, a);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

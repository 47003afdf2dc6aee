// align.hip — intro-offset detection of pipeline.run(auto_align=True): the MI355X path of
// xcorr.find_content_offset (xcorr.py:165-259).  CPU restatement: oracle/refglue.py
// find_content_offset on oracle/ncref.py resample_half / rms_frames.
//
// Per (src, nc) pair, all pairs of a batch at once:
//   1. align_plan_kernel      file layout + per (pair, speed) stretch length and lag count
//   2. align_decimate_kernel  librosa.resample(y, 22050 -> 11025) (scale=False): the
//                             half-band of nc_decim.h, f64 accumulation
//   3. align_env_kernel       librosa.feature.rms(hop 512, frame 2048, centred, zero pad)
//                             -> f64 envelope (xcorr.py:210-211)
//   4. align_stretch_kernel   np.interp of the nc envelope onto int(len / speed) points for
//                             each of the 30 speeds (numpy's linspace / interp arithmetic)
//   5. align_corr_kernel      np.correlate(src_env[:search + n], stretched, 'valid'): one
//                             lag per thread, both operands staged through LDS in tiles
//   6. align_select_kernel    per speed in order: first argmax, window / query energies,
//                             cosine score; strict '>' over speeds (xcorr.py:244-259)
#include <algorithm>

#include "nc_block.h"
#include "nc_decim.h"
#include "nc_engine.h"

namespace nc {

constexpr int AL_HOP = 512, AL_FRAME = 2048;

struct AlignWs {
  int64_t* dec_base;  // [n_files + 1] decimated-signal offsets (64-float aligned)
  int64_t* env_base;  // [n_files + 1] envelope offsets
  int* n_st;          // [pair][speed] stretched length (0: speed skipped)
  int* n_lag;         // [pair][speed] lags searched = search_len + 1 (0: skipped)
  float* dec;
  double* env;
  double* st;         // [pair][speed][st_stride]
  double* corr;       // [pair][speed][lag_stride]
};

__device__ __forceinline__ int64_t al_dec_len(int64_t L) { return (L + 1) / 2; }
__device__ __forceinline__ int64_t al_env_len(int64_t L) { return 1 + al_dec_len(L) / AL_HOP; }

// files are ordered src_0, nc_0, src_1, nc_1, ...
__device__ __forceinline__ int64_t al_file_len(const int64_t* src_len, const int64_t* nc_len, int f) {
  return (f & 1) ? nc_len[f >> 1] : src_len[f >> 1];
}
__device__ __forceinline__ int64_t al_file_off(const int64_t* src_off, const int64_t* nc_off, int f) {
  return (f & 1) ? nc_off[f >> 1] : src_off[f >> 1];
}

__global__ __launch_bounds__(256) void align_plan_kernel(const int64_t* src_len, const int64_t* nc_len, int n_pairs,
                                                         const double* speeds, int n_speeds, int max_off_frames,
                                                         AlignWs w) {
  const int nf = 2 * n_pairs;
  block_prefix_table<256>(nf, w.dec_base,
                          [&](int f) { return (al_dec_len(al_file_len(src_len, nc_len, f)) + 63) & ~63LL; });
  block_prefix_table<256>(nf, w.env_base, [&](int f) { return al_env_len(al_file_len(src_len, nc_len, f)); });
  for (int q = threadIdx.x; q < n_pairs * n_speeds; q += 256) {
    const int p = q / n_speeds, s = q - p * n_speeds;
    const int64_t ns = al_env_len(src_len[p]), nn = al_env_len(nc_len[p]);
    const int64_t n_st = (int64_t)((double)nn / speeds[s]);          // int(len(nc_env) / speed)
    int64_t sl = min((int64_t)max_off_frames, ns - n_st);            // search_len
    const bool ok = n_st >= 4 && n_st < ns && sl > 0;
    w.n_st[q] = ok ? (int)n_st : 0;
    w.n_lag[q] = ok ? (int)(sl + 1) : 0;
  }
}

__global__ __launch_bounds__(256) void align_decimate_kernel(const float* sig, const int64_t* src_off,
                                                             const int64_t* src_len, const int64_t* nc_off,
                                                             const int64_t* nc_len, AlignWs w,
                                                             const double* __restrict__ taps) {
  const int f = blockIdx.y;
  const int64_t L = al_file_len(src_len, nc_len, f), Lout = al_dec_len(L);
  const int64_t m0 = (int64_t)blockIdx.x * DEC_OUT;
  if (m0 >= Lout) return;
  halfband_tile<false>(sig + al_file_off(src_off, nc_off, f), L, w.dec + w.dec_base[f], Lout, m0, taps);
}

// one wave per frame: sqrt(mean over the 2048-sample centred frame of x^2) (squares in f32,
// summed in f64, rounded to f32 like the f32 envelope the reference computes), stored f64
__global__ __launch_bounds__(256) void align_env_kernel(const int64_t* src_len, const int64_t* nc_len, AlignWs w) {
  const int f = blockIdx.y;
  const int64_t Ld = al_dec_len(al_file_len(src_len, nc_len, f));
  const int64_t T = 1 + Ld / AL_HOP;
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const float* x = w.dec + w.dec_base[f];
  const int64_t s0 = t * AL_HOP - AL_FRAME / 2;
  double acc = 0.0;
#pragma unroll 8
  for (int q = 0; q < AL_FRAME / 64; ++q) {
    const int64_t i = s0 + lane + 64 * q;
    const float v = (i >= 0 && i < Ld) ? x[i] : 0.0f;
    acc += (double)(v * v);
  }
  acc = wave_sum(acc);
  if (lane == 0) w.env[w.env_base[f] + t] = (double)sqrtf((float)(acc / (double)AL_FRAME));
}

// np.interp(linspace(0, 1, n_st), linspace(0, 1, n), nc_env): linspace(0, 1, m)[i] = i * (1 / (m - 1)),
// last = 1 exactly; interval j = last xp[j] <= x; slope * (x - xp[j]) + fp[j], no contraction
__device__ __forceinline__ double al_lin(int64_t i, int64_t m, double step) { return i == m - 1 ? 1.0 : (double)i * step; }

__global__ __launch_bounds__(256) void align_stretch_kernel(const int64_t* nc_len, int n_speeds, int st_stride,
                                                            AlignWs w) {
#pragma clang fp contract(off)
  const int s = blockIdx.y, p = blockIdx.z;
  const int q = p * n_speeds + s;
  const int n_st = w.n_st[q];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_st) return;
  const double* fp = w.env + w.env_base[2 * p + 1];
  const int64_t n = al_env_len(nc_len[p]);
  const double step_n = 1.0 / (double)(n_st - 1), step_o = 1.0 / (double)(n - 1);
  const double x = al_lin(i, n_st, step_n);
  double r;
  if (n == 1) {
    r = fp[0];
  } else {
    int64_t j = (int64_t)(x / step_o);
    j = max((int64_t)0, min(j, n - 1));
    while (j + 1 < n && al_lin(j + 1, n, step_o) <= x) ++j;
    while (j > 0 && al_lin(j, n, step_o) > x) --j;
    const double xj = al_lin(j, n, step_o);
    if (j == n - 1 || xj == x) {
      r = fp[j];
    } else {
      const double slope = (fp[j + 1] - fp[j]) / (al_lin(j + 1, n, step_o) - xj);
      r = slope * (x - xj) + fp[j];
    }
  }
  w.st[(size_t)q * st_stride + i] = r;
}

constexpr int AL_TILE = 1024;

__global__ __launch_bounds__(256) void align_corr_kernel(int n_speeds, int st_stride, int lag_stride, AlignWs w) {
  __shared__ double sh_st[AL_TILE];
  __shared__ double sh_src[AL_TILE + 256];
  const int s = blockIdx.y, p = blockIdx.z;
  const int q = p * n_speeds + s;
  const int n_st = w.n_st[q], n_lag = w.n_lag[q];
  const int lag0 = blockIdx.x * 256;
  if (lag0 >= n_lag) return;
  const int lag = lag0 + threadIdx.x;
  const double* src = w.env + w.env_base[2 * p];
  const double* st = w.st + (size_t)q * st_stride;
  double acc = 0.0;
  for (int i0 = 0; i0 < n_st; i0 += AL_TILE) {
    const int nt = min(AL_TILE, n_st - i0);
    __syncthreads();
    for (int u = threadIdx.x; u < nt; u += 256) sh_st[u] = st[i0 + u];
    // src_env[lag0 + i0 + u] for u < nt + 255 (all inside src: lag + i < n_lag - 1 + n_st <= len(src_env))
    for (int u = threadIdx.x; u < nt + 255 && lag0 + i0 + u < n_lag - 1 + n_st; u += 256) sh_src[u] = src[lag0 + i0 + u];
    __syncthreads();
    if (lag < n_lag)
      for (int u = 0; u < nt; ++u) acc = fma(sh_src[threadIdx.x + u], sh_st[u], acc);
  }
  if (lag < n_lag) w.corr[(size_t)q * lag_stride + lag] = acc;
}

__global__ __launch_bounds__(256) void align_select_kernel(int n_speeds, int st_stride, int lag_stride, AlignWs w,
                                                           int* out_peak, int* out_speed, double* out_score) {
  __shared__ BlockScratch<256> bs;
  const int p = blockIdx.x;
  const double* src = w.env + w.env_base[2 * p];
  double best = -1.0;
  int best_s = -1, best_pk = 0;
  for (int s = 0; s < n_speeds; ++s) {
    const int q = p * n_speeds + s;
    const int n_st = w.n_st[q], n_lag = w.n_lag[q];
    if (n_lag == 0) continue;
    const double* corr = w.corr + (size_t)q * lag_stride;
    const double* st = w.st + (size_t)q * st_stride;
    double v = -INFINITY;
    int idx = 0x7fffffff;
    for (int l = threadIdx.x; l < n_lag; l += 256)
      if (np_better(corr[l], l, v, idx)) {
        v = corr[l];
        idx = l;
      }
    block_argmax<256>(v, idx, bs);
    double we = 0.0, qe = 0.0;
    for (int i = threadIdx.x; i < n_st; i += 256) {
      const double a = src[idx + i], b = st[i];
      we += a * a;
      qe += b * b;
    }
    we = block_sum<256>(we, bs);
    qe = block_sum<256>(qe, bs);
    const double denom = sqrt(we * qe);
    const double score = denom > 1e-12 ? v / denom : 0.0;
    if (score > best) {
      best = score;
      best_s = s;
      best_pk = idx;
    }
  }
  if (threadIdx.x == 0) {
    out_peak[p] = best_pk;
    out_speed[p] = best_s;
    out_score[p] = best;
  }
}

static inline size_t al256(size_t n) { return (n + 255) & ~(size_t)255; }

// strides: st_stride >= envelope frames of the longest nc file, lag_stride >= max_off_frames + 1
static void align_strides(int64_t max_len, int max_off_frames, int& st_stride, int& lag_stride) {
  st_stride = (int)(1 + ((max_len + 1) / 2) / AL_HOP);
  lag_stride = max_off_frames + 1;
}

size_t align_ws_bytes(int n_pairs, int n_speeds, int64_t total_len, int64_t max_len, int max_off_frames) {
  int st_stride, lag_stride;
  align_strides(max_len, max_off_frames, st_stride, lag_stride);
  const int nf = 2 * n_pairs;
  const size_t q = (size_t)n_pairs * n_speeds;
  size_t b = al256(sizeof(int64_t) * (nf + 1)) * 2 + al256(sizeof(int) * q) * 2;
  b += al256(sizeof(float) * (size_t)(total_len / 2 + 64 * (int64_t)nf + nf));
  b += al256(sizeof(double) * (size_t)(total_len / 2 / AL_HOP + 2 * (int64_t)nf));
  b += al256(sizeof(double) * q * st_stride) + al256(sizeof(double) * q * lag_stride);
  return b + 4096;
}

int launch_align_offsets(Context& ctx, const float* sig, const int64_t* src_off, const int64_t* src_len,
                         const int64_t* nc_off, const int64_t* nc_len, int n_pairs, const double* speeds,
                         int n_speeds, int max_off_frames, int64_t total_len, int64_t max_len, int* out_peak,
                         int* out_speed, double* out_score, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n_pairs <= 0) return 0;
  if (n_speeds <= 0 || max_off_frames < 0 || max_len <= 0) {
    set_error("align: n_speeds, max_offset_frames and max_len must be positive");
    return -2;
  }
  if (ws_bytes < align_ws_bytes(n_pairs, n_speeds, total_len, max_len, max_off_frames)) {
    set_error("align: workspace too small");
    return -3;
  }
  int st_stride, lag_stride;
  align_strides(max_len, max_off_frames, st_stride, lag_stride);
  const int nf = 2 * n_pairs;
  const size_t q = (size_t)n_pairs * n_speeds;
  char* c = static_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* r = c;
    c += al256(bytes);
    return r;
  };
  AlignWs w;
  w.dec_base = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (nf + 1)));
  w.env_base = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (nf + 1)));
  w.n_st = reinterpret_cast<int*>(take(sizeof(int) * q));
  w.n_lag = reinterpret_cast<int*>(take(sizeof(int) * q));
  w.dec = reinterpret_cast<float*>(take(sizeof(float) * (size_t)(total_len / 2 + 64 * (int64_t)nf + nf)));
  w.env = reinterpret_cast<double*>(take(sizeof(double) * (size_t)(total_len / 2 / AL_HOP + 2 * (int64_t)nf)));
  w.st = reinterpret_cast<double*>(take(sizeof(double) * q * st_stride));
  w.corr = reinterpret_cast<double*>(take(sizeof(double) * q * lag_stride));
  hipLaunchKernelGGL(align_plan_kernel, dim3(1), dim3(256), 0, st, src_len, nc_len, n_pairs, speeds, n_speeds,
                     max_off_frames, w);
  const int64_t max_dec = (max_len + 1) / 2;
  hipLaunchKernelGGL(align_decimate_kernel, dim3((unsigned)((max_dec + DEC_OUT - 1) / DEC_OUT), nf), dim3(256), 0,
                     st, sig, src_off, src_len, nc_off, nc_len, w, ctx.t.halfband);
  const int64_t max_env = 1 + max_dec / AL_HOP;
  hipLaunchKernelGGL(align_env_kernel, dim3((unsigned)((max_env + 3) / 4), nf), dim3(256), 0, st, src_len, nc_len, w);
  hipLaunchKernelGGL(align_stretch_kernel, dim3((unsigned)((st_stride + 255) / 256), n_speeds, n_pairs), dim3(256), 0,
                     st, nc_len, n_speeds, st_stride, w);
  hipLaunchKernelGGL(align_corr_kernel, dim3((unsigned)((lag_stride + 255) / 256), n_speeds, n_pairs), dim3(256), 0,
                     st, n_speeds, st_stride, lag_stride, w);
  hipLaunchKernelGGL(align_select_kernel, dim3(n_pairs), dim3(256), 0, st, n_speeds, st_stride, lag_stride, w,
                     out_peak, out_speed, out_score);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

// ibi.hip — the hop-64 full-signal pass of tempo.estimate_ibis_global
// (tempo.py:120-173): onset_strength(y, hop_length=64) over the whole trimmed
// file, then the tempogram mean (win_length = 2756) that beat_track's tempo
// estimate argmaxes.  Beat tracking itself reuses beat.hip (large variant).
//
// The reference materialises the (2756 x frames) float64 tempogram (1.37 GB for
// a 3-min file, ~27 GB at 60 min) before averaging; here the mean is streamed:
// the autocorrelation of every frame is evaluated by the five sliding f64 sums
// of nc_slide.h, one thread per lag over a 2048-frame tile (tile inputs in
// LDS), each tile writing one 2756-double partial row; a last kernel sums the
// rows of each file in a fixed order (deterministic, no atomics).
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"
#include "nc_slide.h"
#include "stft_args.h"

namespace nc {

// ------------------------------------------------------------------------------ frame indexing
__global__ __launch_bounds__(256) void ibi_plan_kernel(const int64_t* file_len, int n_files, int hop,
                                                        int64_t* frame_base) {
  block_prefix_table<256>(n_files, frame_base, [&](int f) { return 1 + file_len[f] / hop; });
}

__device__ __forceinline__ int find_file(const int64_t* base, int n, int64_t g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (base[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ------------------------------------------------------------------------------ A: per-file max
// (STFT -> mel dB is stft_mel_kernel, stft.hip, in frame_base mode)
__global__ __launch_bounds__(256) void seq_max_kernel(const float* frame_max, const int64_t* frame_base,
                                                      float* seq_max) {
  __shared__ BlockScratch<256> red;
  const int f = blockIdx.x;
  const int64_t b0 = frame_base[f], b1 = frame_base[f + 1];
  float m = -INFINITY;
  for (int64_t g = b0 + threadIdx.x; g < b1; g += 256) m = fmaxf(m, frame_max[g]);
  const double r = block_max((double)m, red);
  if (threadIdx.x == 0) seq_max[f] = (float)r;
}

// ------------------------------------------------------------------------------ B: onset
__global__ __launch_bounds__(256) void ibi_onset_kernel(const float* sdb, const int64_t* frame_base,
                                                        const float* seq_max, int n_files, int64_t total_frames,
                                                        int pad, float* onset) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= total_frames) return;
  const int f = find_file(frame_base, n_files, g);
  const int64_t t = g - frame_base[f];
  float val = 0.0f;
  if (t >= pad) {
    const float c = seq_max[f] - 80.0f;
    const int64_t j = frame_base[f] + (t - pad);
    const float a0 = fmaxf(sdb[j * 128 + lane], c), a1 = fmaxf(sdb[(j + 1) * 128 + lane], c);
    const float b0 = fmaxf(sdb[j * 128 + lane + 64], c), b1 = fmaxf(sdb[(j + 1) * 128 + lane + 64], c);
    const float part = fmaxf(0.0f, a1 - a0) + fmaxf(0.0f, b1 - b0);
    val = wave_sum(part) * (1.0f / 128.0f);
  }
  if (lane == 0) onset[g] = val;
}

// ------------------------------------------------------------------------------ C: tempogram mean
// x_f = ramp_pad(onset_f) (T_f + N floats, at xbase(f) = frame_base[f] + f N), then
// rinv[g] = 1 / ac_t[0] per frame, then the sliding sums of nc_slide.h over
// (lag block, frame block) tiles, then a fixed-order sum of the tile rows.
constexpr int TG_TB = 2048;  // frames per tile
constexpr int TG_KB = 256;   // lags per tile (= threads)

__global__ void tg_pad_kernel(const float* onset, const int64_t* frame_base, int n_files, int64_t total_padded,
                              int N, float* xpad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total_padded) return;
  // file of padded index i: xbase(f) = frame_base[f] + f N
  int lo = 0, hi = n_files - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (frame_base[mid] + (int64_t)mid * N <= i) lo = mid;
    else hi = mid - 1;
  }
  const int f = lo;
  const int64_t base = frame_base[f];
  const int T = (int)(frame_base[f + 1] - base);
  const int u = (int)(i - base - (int64_t)f * N);
  const int p = N / 2;
  const float* on = onset + base;
  float v;
  if (u < p) v = (float)((double)u * ((double)on[0] / (double)p));
  else if (u < p + T) v = on[u - p];
  else v = (float)((double)(p - 1 - (u - p - T)) * ((double)on[T - 1] / (double)p));
  xpad[i] = v;
}

__global__ __launch_bounds__(256) void tg_rinv_kernel(const float* xpad, const int64_t* frame_base, int n_files,
                                                      int64_t total_frames, int N, const double* __restrict__ wsq,
                                                      const int64_t* b0, const int64_t* b1, double* rinv) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= total_frames) return;
  const int f = find_file(frame_base, n_files, g);
  if (b0) {  // only the frames of this rank's tiles
    const int64_t tb = (g - frame_base[f]) / TG_TB;
    if (tb < b0[f] || tb >= b1[f]) return;
  }
  const float* x = xpad + g + (int64_t)f * N;  // xbase(f) + t
  double s = 0.0;
  for (int j = 0; j < N; ++j) {
    const double v = (double)x[j];
    s = fma(wsq[j], v * v, s);
  }
  rinv[g] = tg_rinv(s);
}

struct TgSlideArgs {
  const float* xpad;
  const double* rinv;
  const int64_t* frame_base;
  int N;
  int n_tblk;     // tiles per file along frames (max over files)
  const int64_t* b0 = nullptr;  // nullable [n_files]: only tiles [b0, b1) of each file
  const int64_t* b1 = nullptr;
  double* slab;   // [n_files][n_tblk][N]
  unsigned long long* span = nullptr;  // nc_profile execution span (nc_device.h)
};

__global__ __launch_bounds__(TG_KB) void tg_slide_kernel(TgSlideArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sh_r = reinterpret_cast<double*>(smem);         // [TG_TB]
  float* sh_x = reinterpret_cast<float*>(sh_r + TG_TB);   // [TG_TB + N]
  const int f = blockIdx.z, tb = blockIdx.y;
  const int64_t base = a.frame_base[f];
  const int T = (int)(a.frame_base[f + 1] - base);
  const int t0 = tb * TG_TB;
  if (t0 >= T || (a.b0 && (tb < a.b0[f] || tb >= a.b1[f]))) return;
  const int t1 = min(T, t0 + TG_TB);
  const int N = a.N;
  const float* xf = a.xpad + base + (int64_t)f * N + t0;
  for (int i = threadIdx.x; i < t1 - t0 + N; i += TG_KB) sh_x[i] = xf[i];
  for (int i = threadIdx.x; i < t1 - t0; i += TG_KB) sh_r[i] = a.rinv[base + t0 + i];
  __syncthreads();
  // lags k and N-1-k per thread (two interleaved recurrences, balanced start-up sums)
  const int k = blockIdx.x * TG_KB + threadIdx.x;
  if (k >= (N + 1) / 2) return;
  auto xl = [&](int i) { return sh_x[i]; };
  auto rl = [&](int t) { return sh_r[t]; };
  const int kb = N - 1 - k;
  double sa, sb;
  slide_lag_sum2(xl, rl, N, k, kb, 0, t1 - t0, sa, sb);
  double* row = a.slab + ((size_t)f * a.n_tblk + tb) * N;
  row[k] = sa;
  if (kb != k) row[kb] = sb;
}

__global__ void tg_reduce_kernel(const double* slab, const int64_t* frame_base, int n_tblk, int N, double* tg_out) {
  const int f = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  const int64_t T = frame_base[f + 1] - frame_base[f];
  const int nt = (int)((T + TG_TB - 1) / TG_TB);
  double s = 0.0;
  for (int b = 0; b < nt; ++b) s += slab[((size_t)f * n_tblk + b) * N + k];
  tg_out[(size_t)f * N + k] = s / (double)T;
}

// ------------------------------------------------------------------------------ D: one rank's share
// The window-sharded runs split the hop-64 pass of a file over the ranks (SURVEY.md §8e
// C2-C4): rank r computes the onsets of its frames [t0, t1) -- the mel dB rows they need,
// [t0 - pad, t1 - pad + 1), then the onsets against the file's GLOBAL dB maximum (the
// power_to_db top_db clamp, all-reduced with MAX between the two calls) -- and the tempogram
// partial rows of its 2048-frame tiles [b0, b1) from the gathered full onset; the fixed-order
// sum of every tile's row (tg_reduce_kernel) then equals the one-GPU result bit for bit.
__global__ __launch_bounds__(256) void ibi_range_plan_kernel(const int64_t* file_len, const int64_t* t0,
                                                             const int64_t* t1, int n_files, int hop, int pad,
                                                             int64_t* row0, int64_t* row_base, int64_t* obase) {
  // rows [row0, row1) of file f: its STFT frames [t0 - pad, t1 - pad + 1) within [0, T_f);
  // the share that ends the file takes every row up to T_f: rows T_f - pad + 1 .. T_f - 1
  // feed no onset but do feed the file's dB maximum (the top_db reference all-reduced by C2),
  // as over the whole file on one GPU (sharded._ibi_mel_rows: the same bounds)
  auto rows = [&](int f) -> int64_t {
    const int64_t T = 1 + file_len[f] / hop;
    const int64_t r0 = max((int64_t)0, t0[f] - pad);
    const int64_t r1 = (t1[f] >= T && t1[f] > t0[f]) ? T : min(T, t1[f] - pad + 1);
    return r1 > r0 ? r1 - r0 : 0;
  };
  block_prefix_table<256>(n_files, row_base, rows);
  block_prefix_table<256>(n_files, obase, [&](int f) { return t1[f] > t0[f] ? t1[f] - t0[f] : (int64_t)0; });
  __syncthreads();
  for (int f = threadIdx.x; f < n_files; f += 256) row0[f] = max((int64_t)0, t0[f] - pad);
}

__global__ __launch_bounds__(256) void ibi_onset_range_kernel(const float* sdb, const int64_t* row_base,
                                                              const int64_t* row0, const int64_t* t0,
                                                              const int64_t* obase, const float* gmax, int n_files,
                                                              int64_t total_out, int pad, float* onset) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= total_out) return;
  const int f = find_file(obase, n_files, g);
  const int64_t t = t0[f] + (g - obase[f]);
  float val = 0.0f;
  if (t >= pad) {
    const float c = gmax[f] - 80.0f;
    const int64_t j = row_base[f] + (t - pad - row0[f]);
    const float a0 = fmaxf(sdb[j * 128 + lane], c), a1 = fmaxf(sdb[(j + 1) * 128 + lane], c);
    const float b0 = fmaxf(sdb[j * 128 + lane + 64], c), b1 = fmaxf(sdb[(j + 1) * 128 + lane + 64], c);
    const float part = fmaxf(0.0f, a1 - a0) + fmaxf(0.0f, b1 - b0);
    val = wave_sum(part) * (1.0f / 128.0f);
  }
  if (lane == 0) onset[g] = val;
}

// ------------------------------------------------------------------------------ host
static inline size_t a256(size_t n) { return (n + 255) & ~(size_t)255; }

size_t ibi_range_ws_bytes(int n_files, int64_t total_rows) {
  return 4 * a256(sizeof(int64_t) * (n_files + 1)) + a256(sizeof(float) * (size_t)total_rows) +
         a256(sizeof(float) * (size_t)total_rows * 128) + 4096;
}

struct IbiRangeWs {
  int64_t *row0, *row_base, *obase;
  float *fmax_, *sdb;
};
static IbiRangeWs ibi_range_ws(void* ws, int n_files, int64_t total_rows) {
  char* p = static_cast<char*>(ws);
  IbiRangeWs w;
  w.row0 = reinterpret_cast<int64_t*>(p);
  p += a256(sizeof(int64_t) * (n_files + 1));
  w.row_base = reinterpret_cast<int64_t*>(p);
  p += a256(sizeof(int64_t) * (n_files + 1));
  w.obase = reinterpret_cast<int64_t*>(p);
  p += 2 * a256(sizeof(int64_t) * (n_files + 1));
  w.fmax_ = reinterpret_cast<float*>(p);
  p += a256(sizeof(float) * (size_t)total_rows);
  w.sdb = reinterpret_cast<float*>(p);
  return w;
}

int launch_ibi_mel_range(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                         int n_files, const int64_t* t0, const int64_t* t1, int hop, int64_t total_rows,
                         float* max_out, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n_files <= 0) return 0;
  if (ws_bytes < ibi_range_ws_bytes(n_files, total_rows)) {
    set_error("ibi_mel_range: workspace too small");
    return -3;
  }
  IbiRangeWs w = ibi_range_ws(ws, n_files, total_rows);
  const int pad = 1 + kNFFT / (2 * hop);
  hipLaunchKernelGGL(ibi_range_plan_kernel, dim3(1), dim3(256), 0, st, file_len, t0, t1, n_files, hop, pad, w.row0,
                     w.row_base, w.obase);
  if (total_rows > 0) {
    StftMelArgs s{};
    s.sig = sig;
    s.seq_off = file_off;
    s.seq_len = file_len;
    s.frame_base = w.row_base;
    s.seq_t0 = w.row0;
    s.n_seq = n_files;
    s.total_frames = total_rows;
    s.hop = hop;
    s.sdb = w.sdb;
    s.frame_max = w.fmax_;
    s.frame_energy = nullptr;
    const int rc = launch_stft_mel(ctx, s, st);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(seq_max_kernel, dim3(n_files), dim3(256), 0, st, w.fmax_, w.row_base, max_out);
  NC_HIP(hipGetLastError());
  return 0;
}

int launch_ibi_onset_range(int n_files, const int64_t* t0, int hop, int64_t total_out, const float* gmax,
                           float* onset_out, void* ws, int64_t total_rows, hipStream_t st) {
  if (n_files <= 0 || total_out <= 0) return 0;
  IbiRangeWs w = ibi_range_ws(ws, n_files, total_rows);
  hipLaunchKernelGGL(ibi_onset_range_kernel, dim3((unsigned)((total_out + 3) / 4)), dim3(256), 0, st, w.sdb,
                     w.row_base, w.row0, t0, w.obase, gmax, n_files, total_out, 1 + kNFFT / (2 * hop), onset_out);
  NC_HIP(hipGetLastError());
  return 0;
}

size_t ibi_onset_ws_bytes(int n_files, int64_t total_frames) {
  return a256(sizeof(int64_t) * (n_files + 1)) + a256(sizeof(float) * n_files) +
         a256(sizeof(float) * (size_t)total_frames) + a256(sizeof(float) * (size_t)total_frames * 128) + 4096;
}

int launch_ibi_onset(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                     int64_t total_frames, int hop, float* onset_out, int64_t* frame_base_out, void* ws,
                     size_t ws_bytes, hipStream_t st) {
  if (n_files <= 0) return 0;
  if (ws_bytes < ibi_onset_ws_bytes(n_files, total_frames)) {
    set_error("ibi_onset: workspace too small");
    return -3;
  }
  char* p = static_cast<char*>(ws);
  int64_t* fb = frame_base_out ? frame_base_out : reinterpret_cast<int64_t*>(p);
  p += a256(sizeof(int64_t) * (n_files + 1));
  float* smax = reinterpret_cast<float*>(p);
  p += a256(sizeof(float) * n_files);
  float* fmax_ = reinterpret_cast<float*>(p);
  p += a256(sizeof(float) * (size_t)total_frames);
  float* sdb = reinterpret_cast<float*>(p);
  hipLaunchKernelGGL(ibi_plan_kernel, dim3(1), dim3(256), 0, st, file_len, n_files, hop, fb);
  StftMelArgs s{};
  s.sig = sig;
  s.seq_off = file_off;
  s.seq_len = file_len;
  s.frame_base = fb;
  s.n_seq = n_files;
  s.total_frames = total_frames;
  s.hop = hop;
  s.sdb = sdb;
  s.frame_max = fmax_;
  s.frame_energy = nullptr;
  int rc = launch_stft_mel(ctx, s, st);
  if (rc) return rc;
  hipLaunchKernelGGL(seq_max_kernel, dim3(n_files), dim3(256), 0, st, fmax_, fb, smax);
  const unsigned blocks = (unsigned)((total_frames + 3) / 4);
  hipLaunchKernelGGL(ibi_onset_kernel, dim3(blocks), dim3(256), 0, st, sdb, fb, smax, n_files, total_frames,
                     1 + kNFFT / (2 * hop), onset_out);
  NC_HIP(hipGetLastError());
  return 0;
}

static int tg_acw(const Context& ctx, int hop) { return hop == 64 ? ctx.t.ac64 : (hop == 512 ? ctx.t.ac512 : 0); }

size_t ibi_tg_ws_bytes(const Context& ctx, int n_files, int64_t total_frames, int max_frames, int hop) {
  const int N = tg_acw(ctx, hop);
  const int n_tblk = (max_frames + TG_TB - 1) / TG_TB;
  return a256(sizeof(float) * ((size_t)total_frames + (size_t)n_files * N)) +
         a256(sizeof(double) * (size_t)total_frames) + a256(sizeof(double) * (size_t)n_files * n_tblk * N) + 256;
}

int launch_ibi_tempogram_tiles(Context& ctx, const float* onset, const int64_t* frame_base, int n_files,
                               int64_t total_frames, int max_frames, int hop, const int64_t* b0, const int64_t* b1,
                               double* slab_out, double* tg_out, void* ws, size_t ws_bytes, hipStream_t st);

int launch_ibi_tempogram(Context& ctx, const float* onset, const int64_t* frame_base, int n_files,
                         int64_t total_frames, int max_frames, int hop, double* tg_out, void* ws, size_t ws_bytes,
                         hipStream_t st) {
  return launch_ibi_tempogram_tiles(ctx, onset, frame_base, n_files, total_frames, max_frames, hop, nullptr, nullptr,
                                    nullptr, tg_out, ws, ws_bytes, st);
}

int launch_ibi_tempogram_reduce(Context& ctx, const double* slab, const int64_t* frame_base, int n_files,
                                int max_frames, int hop, double* tg_out, hipStream_t st) {
  const int N = tg_acw(ctx, hop);
  if (N <= 0 || n_files <= 0 || max_frames <= 0) {
    set_error("ibi_tempogram_reduce: bad shape");
    return -2;
  }
  const int n_tblk = (max_frames + TG_TB - 1) / TG_TB;
  hipLaunchKernelGGL(tg_reduce_kernel, dim3((N + 255) / 256, n_files), dim3(256), 0, st, slab, frame_base, n_tblk,
                     N, tg_out);
  NC_HIP(hipGetLastError());
  return 0;
}

// slab_out (nullable): the caller's [n_files][n_tblk][N] rows instead of the workspace's;
// tg_out (nullable): the reduce (every tile must then be in the slab)
int launch_ibi_tempogram_tiles(Context& ctx, const float* onset, const int64_t* frame_base, int n_files,
                               int64_t total_frames, int max_frames, int hop, const int64_t* b0, const int64_t* b1,
                               double* slab_out, double* tg_out, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n_files <= 0 || total_frames <= 0) return 0;
  const int N = tg_acw(ctx, hop);
  if (N <= 0 || (N & 1)) {
    set_error("ibi_tempogram: unsupported hop");
    return -2;
  }
  if (max_frames <= 0 || (int64_t)max_frames > total_frames) {
    set_error("ibi_tempogram: max_frames out of range");
    return -2;
  }
  if (ws_bytes < ibi_tg_ws_bytes(ctx, n_files, total_frames, max_frames, hop)) {
    set_error("ibi_tempogram: workspace too small");
    return -3;
  }
  const int n_tblk = (max_frames + TG_TB - 1) / TG_TB;
  const int64_t total_padded = total_frames + (int64_t)n_files * N;
  char* p = static_cast<char*>(ws);
  float* xpad = reinterpret_cast<float*>(p);
  p += a256(sizeof(float) * (size_t)total_padded);
  double* rinv = reinterpret_cast<double*>(p);
  p += a256(sizeof(double) * (size_t)total_frames);
  double* slab = slab_out ? slab_out : reinterpret_cast<double*>(p);
  hipLaunchKernelGGL(tg_pad_kernel, dim3((unsigned)((total_padded + 255) / 256)), dim3(256), 0, st, onset,
                     frame_base, n_files, total_padded, N, xpad);
  hipLaunchKernelGGL(tg_rinv_kernel, dim3((unsigned)((total_frames + 255) / 256)), dim3(256), 0, st, xpad,
                     frame_base, n_files, total_frames, N, hop == 64 ? ctx.t.wsq64 : ctx.t.wsq512, b0, b1, rinv);
  TgSlideArgs a;
  a.xpad = xpad;
  a.rinv = rinv;
  a.frame_base = frame_base;
  a.N = N;
  a.n_tblk = n_tblk;
  a.b0 = b0;
  a.b1 = b1;
  a.slab = slab;
  const size_t lds = TG_TB * sizeof(double) + (size_t)(TG_TB + N) * sizeof(float);
  {
    KTimer kt_(ctx, "tg_slide", st);
    a.span = kt_.span();
    hipLaunchKernelGGL(tg_slide_kernel, dim3(((N + 1) / 2 + TG_KB - 1) / TG_KB, n_tblk, n_files), dim3(TG_KB), lds, st,
                     a);
  }
  if (tg_out)
    hipLaunchKernelGGL(tg_reduce_kernel, dim3((N + 255) / 256, n_files), dim3(256), 0, st, slab, frame_base, n_tblk,
                       N, tg_out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

// ibi.hip — the hop-64 full-signal pass of tempo.estimate_ibis_global
// (tempo.py:120-173): onset_strength(y, hop_length=64) over the whole trimmed
// file, then the tempogram mean (win_length = 2756) that beat_track's tempo
// estimate argmaxes.  Beat tracking itself reuses beat.hip (large variant).
//
// The reference materialises the (2756 x frames) float64 tempogram (1.37 GB for
// a 3-min file, ~27 GB at 60 min) before averaging; here the mean is streamed:
// each workgroup owns a contiguous run of frames, runs two 4096-point complex
// FFTs per frame across its 4 waves (8192-point real autocorrelation,
// 34.8 KB LDS), keeps the normalised lags in f64 registers (12 per thread) and
// writes one 2756-double partial row; a second kernel sums the rows of each
// file in a fixed order (deterministic, no atomics).
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

// ------------------------------------------------------------------------------ frame indexing
__global__ void ibi_plan_kernel(const int64_t* file_len, int n_files, int hop, int64_t* frame_base) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t acc = 0;
  for (int f = 0; f < n_files; ++f) {
    frame_base[f] = acc;
    acc += 1 + file_len[f] / hop;
  }
  frame_base[n_files] = acc;
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

// ------------------------------------------------------------------------------ A: STFT -> mel dB
struct IbiSdbArgs {
  const float* sig;
  const int64_t* file_off;
  const int64_t* file_len;
  const int64_t* frame_base;
  int n_files;
  int64_t total_frames;
  int hop;
  float* sdb;      // [total_frames][128]
  int* fmax_ord;   // [n_files] order-preserving int of the per-file max
  const float2* tw;
  const float* hann2048;
  const int* mel_lo;
  const int* mel_len;
  const int* mel_off;
  const float* mel_w;
};

__global__ __launch_bounds__(256) void ibi_sdb_kernel(IbiSdbArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float2* fftbuf = reinterpret_cast<float2*>(smem) + wave * LdsSize<1024>::value;
  const int64_t g = (int64_t)blockIdx.x * 4 + wave;
  if (g >= a.total_frames) return;
  const int f = find_file(a.frame_base, a.n_files, g);
  const int64_t t = g - a.frame_base[f];
  const float* x = a.sig + a.file_off[f];
  const int64_t L = a.file_len[f];
  const int64_t s0 = t * a.hop - 1024;
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
  float lmax = -INFINITY;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int b = h == 0 ? lane : 127 - lane;
    const int lo = a.mel_lo[b], len = a.mel_len[b], off = a.mel_off[b];
    float acc = 0.0f;
    for (int j = 0; j < len; ++j) acc = fmaf(a.mel_w[off + j], pw[lo + j], acc);
    const float db = 10.0f * log10f(fmaxf(1e-10f, acc));
    a.sdb[g * 128 + b] = db;
    lmax = fmaxf(lmax, db);
  }
  lmax = wave_max(lmax);
  if (lane == 0) atomicMax(&a.fmax_ord[f], f2ord(lmax));
}

// ------------------------------------------------------------------------------ B: onset
__global__ __launch_bounds__(256) void ibi_onset_kernel(const float* sdb, const int64_t* frame_base,
                                                        const int* fmax_ord, int n_files, int64_t total_frames,
                                                        int pad, float* onset) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= total_frames) return;
  const int f = find_file(frame_base, n_files, g);
  const int64_t t = g - frame_base[f];
  float val = 0.0f;
  if (t >= pad) {
    const float c = ord2f(fmax_ord[f]) - 80.0f;
    const int64_t j = frame_base[f] + (t - pad);
    const float a0 = fmaxf(sdb[j * 128 + lane], c), a1 = fmaxf(sdb[(j + 1) * 128 + lane], c);
    const float b0 = fmaxf(sdb[j * 128 + lane + 64], c), b1 = fmaxf(sdb[(j + 1) * 128 + lane + 64], c);
    const float part = fmaxf(0.0f, a1 - a0) + fmaxf(0.0f, b1 - b0);
    val = wave_sum(part) * (1.0f / 128.0f);
  }
  if (lane == 0) onset[g] = val;
}

// ------------------------------------------------------------------------------ C: tempogram partials
constexpr int IT = 256;       // threads per workgroup (one 4096-point complex FFT)
constexpr int IBI_NQ = 6;     // lag pairs per thread: n = tid + 256 q, 2n+1 < acw <= 3072

struct IbiTgArgs {
  const float* onset;
  const int64_t* frame_base;
  int n_files;
  int blocks_per_file;
  int acw;
  const float2* tw;
  const float* wac;
  double* slab;  // [n_files][blocks_per_file][acw]
};

__global__ __launch_bounds__(IT) void ibi_tg_kernel(IbiTgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[IT / 64];
  float2* buf = reinterpret_cast<float2*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int f = blockIdx.y, blk = blockIdx.x;
  const int64_t base = a.frame_base[f];
  const int T = (int)(a.frame_base[f + 1] - base);
  const float* on = a.onset + base;
  const int acw = a.acw, p = acw / 2;
  const int t0 = (int)((int64_t)T * blk / a.blocks_per_file);
  const int t1 = (int)((int64_t)T * (blk + 1) / a.blocks_per_file);
  const double st0 = (double)on[0] / (double)p, stl = (double)on[T - 1] / (double)p;
  auto opad = [&](int i) -> float {
    if (i < p) return (float)((double)i * st0);
    if (i < p + T) return on[i - p];
    return (float)((double)(p - 1 - (i - p - T)) * stl);
  };
  double acc[IBI_NQ][2];
#pragma unroll
  for (int q = 0; q < IBI_NQ; ++q) acc[q][0] = acc[q][1] = 0.0;

  for (int t = t0; t < t1; ++t) {
    FftIn<4096, IT> in;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j0 = 2 * (tid + IT * r);
      const float v0 = j0 < acw ? opad(t + j0) * a.wac[j0] : 0.0f;
      const float v1 = j0 + 1 < acw ? opad(t + j0 + 1) * a.wac[j0 + 1] : 0.0f;
      in[0][r] = make_float2(v0, v1);
    }
    block_fft<4096, IT>(in, buf, a.tw, tid);
    float pk[9], pn[9];
#pragma unroll
    for (int m = 0; m < 9; ++m) {
      const int k = tid + IT * m;
      if (k <= 2048) {
        float2 X, XN;
        rfft_split(buf, a.tw, 4096, k, X, XN);
        pk[m] = fmaf(X.x, X.x, X.y * X.y);
        pn[m] = fmaf(XN.x, XN.x, XN.y * XN.y);
      }
    }
    __syncthreads();
    float* pw = reinterpret_cast<float*>(buf);
#pragma unroll
    for (int m = 0; m < 9; ++m) {
      const int k = tid + IT * m;
      if (k <= 2048) {
        pw[k] = pk[m];
        pw[4096 - k] = pn[m];
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = tid + IT * r;
      const float Pa = pw[n], Pb = pw[4096 - n];
      const float E = 0.5f * (Pa + Pb), Od = 0.5f * (Pa - Pb);
      const float2 wv = a.tw[n & 8191];  // exp(-2 pi i n / 8192) = (cos, -sin)
      const float cs = wv.x, sn = -wv.y;
      in[0][r] = make_float2(E - Od * sn, -(Od * cs));
    }
    block_fft<4096, IT>(in, buf, a.tw, tid);
    float av[IBI_NQ][2];
    float mx = 0.0f;
#pragma unroll
    for (int q = 0; q < IBI_NQ; ++q) {
      const int n = tid + IT * q;
      av[q][0] = av[q][1] = 0.0f;
      if (2 * n < acw) {
        const float2 y = buf[lpad(n)];
        av[q][0] = y.x;
        av[q][1] = (2 * n + 1 < acw) ? -y.y : 0.0f;
      }
      mx = fmaxf(mx, fmaxf(fabsf(av[q][0]), fabsf(av[q][1])));
    }
    mx = wave_max(mx);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const double inv = (mx < 1.17549435e-38f) ? 1.0 : 1.0 / (double)mx;
#pragma unroll
    for (int q = 0; q < IBI_NQ; ++q) {
      acc[q][0] += (double)av[q][0] * inv;
      acc[q][1] += (double)av[q][1] * inv;
    }
    __syncthreads();
  }
  double* row = a.slab + ((size_t)f * a.blocks_per_file + blk) * acw;
#pragma unroll
  for (int q = 0; q < IBI_NQ; ++q) {
    const int n = tid + IT * q;
    if (2 * n < acw) row[2 * n] = acc[q][0];
    if (2 * n + 1 < acw) row[2 * n + 1] = acc[q][1];
  }
}

__global__ void ibi_tg_reduce_kernel(const double* slab, const int64_t* frame_base, int blocks_per_file, int acw,
                                     double* tg_out) {
  const int f = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= acw) return;
  double s = 0.0;
  for (int b = 0; b < blocks_per_file; ++b) s += slab[((size_t)f * blocks_per_file + b) * acw + k];
  const double T = (double)(frame_base[f + 1] - frame_base[f]);
  tg_out[(size_t)f * acw + k] = s / T;
}

// ------------------------------------------------------------------------------ host
static inline size_t a256(size_t n) { return (n + 255) & ~(size_t)255; }

size_t ibi_onset_ws_bytes(int n_files, int64_t total_frames) {
  return a256(sizeof(int64_t) * (n_files + 1)) + a256(sizeof(int) * n_files) +
         a256(sizeof(float) * (size_t)total_frames * 128) + 4096;
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
  int* fmax = reinterpret_cast<int*>(p);
  p += a256(sizeof(int) * n_files);
  float* sdb = reinterpret_cast<float*>(p);
  hipLaunchKernelGGL(ibi_plan_kernel, dim3(1), dim3(64), 0, st, file_len, n_files, hop, fb);
  NC_HIP(hipMemsetAsync(fmax, 0x80, sizeof(int) * n_files, st));  // very negative ordered ints
  IbiSdbArgs a;
  a.sig = sig;
  a.file_off = file_off;
  a.file_len = file_len;
  a.frame_base = fb;
  a.n_files = n_files;
  a.total_frames = total_frames;
  a.hop = hop;
  a.sdb = sdb;
  a.fmax_ord = fmax;
  a.tw = ctx.t.tw;
  a.hann2048 = ctx.t.hann2048;
  a.mel_lo = ctx.t.mel_lo;
  a.mel_len = ctx.t.mel_len;
  a.mel_off = ctx.t.mel_off;
  a.mel_w = ctx.t.mel_w;
  const unsigned blocks = (unsigned)((total_frames + 3) / 4);
  hipLaunchKernelGGL(ibi_sdb_kernel, dim3(blocks), dim3(256), 4 * LdsSize<1024>::value * sizeof(float2), st, a);
  hipLaunchKernelGGL(ibi_onset_kernel, dim3(blocks), dim3(256), 0, st, sdb, fb, fmax, n_files, total_frames,
                     1 + kNFFT / (2 * hop), onset_out);
  NC_HIP(hipGetLastError());
  return 0;
}

int ibi_blocks_per_file(const Context& ctx, int n_files) {
  // ~4 workgroups per CU over the whole batch
  const int target = 4 * ctx.num_cu;
  return std::max(1, std::min(512, target / std::max(1, n_files)));
}

size_t ibi_tg_ws_bytes(const Context& ctx, int n_files, int acw) {
  return a256(sizeof(double) * (size_t)n_files * ibi_blocks_per_file(ctx, n_files) * acw) + 256;
}

int launch_ibi_tempogram(Context& ctx, const float* onset, const int64_t* frame_base, int n_files, int hop,
                         double* tg_out, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n_files <= 0) return 0;
  const int acw = hop == 64 ? ctx.t.ac64 : (hop == 512 ? ctx.t.ac512 : 0);
  const float* wac = hop == 64 ? ctx.t.hann_ac64 : ctx.t.hann_ac512;
  if (acw <= 0 || 2 * acw - 1 > 8192 || acw > 2 * IT * IBI_NQ) {
    set_error("ibi_tempogram: unsupported hop");
    return -2;
  }
  if (ws_bytes < ibi_tg_ws_bytes(ctx, n_files, acw)) {
    set_error("ibi_tempogram: workspace too small");
    return -3;
  }
  IbiTgArgs a;
  a.onset = onset;
  a.frame_base = frame_base;
  a.n_files = n_files;
  a.blocks_per_file = ibi_blocks_per_file(ctx, n_files);
  a.acw = acw;
  a.tw = ctx.t.tw;
  a.wac = wac;
  a.slab = static_cast<double*>(ws);
  hipLaunchKernelGGL(ibi_tg_kernel, dim3(a.blocks_per_file, n_files), dim3(IT),
                     LdsSize<4096>::value * sizeof(float2), st, a);
  hipLaunchKernelGGL(ibi_tg_reduce_kernel, dim3((acw + 255) / 256, n_files), dim3(256), 0, st, a.slab, frame_base,
                     a.blocks_per_file, acw, tg_out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

// resample.hip — rational-ratio polyphase resampler for inputs that are not at
// 22 050 Hz (io.load_audio, io.py:44-55: librosa.load(path, sr=22050) resamples at
// load).  The reference resamples with libsoxr 'soxr_hq', which is absent here and
// cannot be bit-matched; the engine's documented stand-in is
// scipy.signal.resample_poly(x, up, down) with its default Kaiser(5.0) FIR, and this
// kernel reproduces it BIT FOR BIT in f64:
//   y[m'] = upfirdn(h, x, up, down)[m' + pre_remove],  m' < n_out,
//   upfirdn output m: x_idx = floor(m down / up), phase p = (m down) mod up,
//   acc = sum over i = hpp-1 .. 0 (oldest input first) of x[x_idx - i] * h[p + i up],
// with scipy's _upfirdn_apply order: left out-of-range taps skipped while
// x_idx < len_x, every tap (zeros included) added once x_idx >= len_x (the flush
// loop), products and sums rounded separately (no FMA contraction).
//
// MI355X layout: one output per thread, 256 outputs per workgroup; the input span of
// the workgroup (256 down / up + hpp samples) and the f64 filter are staged through
// LDS once (dynamic LDS sized to the ratio), so the hpp-fold reuse of every input
// sample and every tap is served from LDS.  The f64 sum is one dependent chain per
// output (scipy's order, no reassociation), so latency is hidden by occupancy.  Files of one (up, down) ratio share a
// launch (grid.y = file).
#include <algorithm>

#include "nc_engine.h"

namespace nc {

constexpr int RS_THREADS = 256;
constexpr int RS_LDS_MAX = 48 * 1024;  // dynamic LDS cap: filter (f64) + input span (f32)

__global__ __launch_bounds__(RS_THREADS) void resample_poly_kernel(
    const float* __restrict__ x_all, const int64_t* in_off, const int64_t* in_len, float* __restrict__ y_all,
    const int64_t* out_off, const int64_t* out_len, const double* __restrict__ h_g, int hpp, int up, int down,
    int64_t pre_remove, int h_staged, int tile_cap) {
  extern __shared__ double rs_smem[];
  double* h_s = rs_smem;                                        // [h_len] when h_staged
  float* tile = reinterpret_cast<float*>(rs_smem + (h_staged ? hpp * up : 0));  // [tile_cap]
  const int f = blockIdx.y;
  const int64_t n_out = out_len[f];
  const int64_t m0 = (int64_t)blockIdx.x * RS_THREADS;
  if (m0 >= n_out) return;
  const int64_t len_x = in_len[f];
  const float* x = x_all + in_off[f];
  float* y = y_all + out_off[f];

  // input span of this workgroup: [lo, hi]
  const int64_t m_last = min(n_out, m0 + RS_THREADS) - 1 + pre_remove;
  const int64_t lo = (m0 + pre_remove) * down / up - (hpp - 1);
  const int64_t hi = m_last * down / up;
  const bool staged = hi - lo + 1 <= tile_cap;
  const int h_len = hpp * up;
  const double* h = h_g;
  if (h_staged) {
    for (int i = threadIdx.x; i < h_len; i += RS_THREADS) h_s[i] = h_g[i];
    h = h_s;
  }
  if (staged) {
    for (int64_t i = threadIdx.x; i <= hi - lo; i += RS_THREADS) {
      const int64_t xi = lo + i;
      tile[i] = (xi >= 0 && xi < len_x) ? x[xi] : 0.0f;
    }
  }
  __syncthreads();

  const int64_t mo = m0 + threadIdx.x;
  if (mo >= n_out) return;
  const int64_t m = mo + pre_remove;
  const int64_t t = m * down;
  const int64_t x_idx = t / up;
  const int p = (int)(t - x_idx * up);
  const bool flush = x_idx >= len_x;
  const double* hp = h + p;
  double acc = 0.0;
  if (staged && !flush && x_idx >= hpp - 1) {
    // interior output (every tap in range, input span in LDS): 32-bit indices, no branches
    const float* tb = tile + (int)(x_idx - lo);
#pragma unroll 6
    for (int i = hpp - 1; i >= 0; --i) acc = __dadd_rn(acc, __dmul_rn((double)tb[-i], hp[i * up]));
  } else {
    for (int i = hpp - 1; i >= 0; --i) {
      const int64_t xi = x_idx - i;
      if (!flush && xi < 0) continue;  // zero-padded left edge: scipy skips these taps
      const double hv = hp[(int64_t)i * up];
      double xv;
      if (xi < 0 || xi >= len_x) xv = 0.0;
      else xv = (double)(staged ? tile[xi - lo] : x[xi]);
      acc = __dadd_rn(acc, __dmul_rn(xv, hv));
    }
  }
  y[mo] = (float)acc;
}

int launch_resample_poly(const float* x, const int64_t* in_off, const int64_t* in_len, int n_files,
                         float* y, const int64_t* out_off, const int64_t* out_len, int64_t max_out,
                         const double* h, int h_len, int up, int down, int64_t pre_remove, hipStream_t st) {
  if (n_files <= 0 || max_out <= 0) return 0;
  if (up < 1 || down < 1 || h_len < up || h_len % up != 0 || pre_remove < 0) {
    set_error("resample_poly: need up, down >= 1, a filter padded to a multiple of up, pre_remove >= 0");
    return -2;
  }
  const int hpp = h_len / up;
  // LDS sized to this ratio: the filter when it fits, and one workgroup's input span
  // (RS_THREADS down / up + hpp samples) — small enough to keep 8 workgroups per CU
  const int64_t span = (int64_t)RS_THREADS * down / up + hpp + 2;
  const int h_staged = (size_t)h_len * sizeof(double) + 1024 <= RS_LDS_MAX ? 1 : 0;
  const size_t h_bytes = h_staged ? (size_t)h_len * sizeof(double) : 0;
  const int tile_cap = (int)std::max<int64_t>(0, std::min<int64_t>(span, (RS_LDS_MAX - h_bytes) / sizeof(float)));
  const size_t lds = h_bytes + (size_t)tile_cap * sizeof(float);
  const dim3 grid((unsigned)((max_out + RS_THREADS - 1) / RS_THREADS), (unsigned)n_files);
  hipLaunchKernelGGL(resample_poly_kernel, grid, dim3(RS_THREADS), lds, st, x, in_off, in_len, y, out_off, out_len,
                     h, hpp, up, down, pre_remove, h_staged, tile_cap);
  NC_HIP(hipGetLastError());
  return 0;
}

// 16-bit PCM -> f32 (io.load_audio of a mono 16-bit WAV, io.py:44-55: soundfile scales sample k
// to k / 32768, exact in f32).  The host uploads the file's own 2-byte samples (half the bytes of
// f32 over PCIe) and this kernel widens them in HBM.  HBM-bound: each thread reads 16 B (8
// samples) and writes 32 B; a grid-stride loop over the buffer.
__global__ __launch_bounds__(256) void pcm16_to_f32_kernel(const int16_t* __restrict__ x, int64_t n,
                                                           float* __restrict__ y) {
  const int64_t n8 = n >> 3;
  const float s = 1.0f / 32768.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int4 v = reinterpret_cast<const int4*>(x)[i];
    const int w[4] = {v.x, v.y, v.z, v.w};
    float4 lo, hi;
    lo.x = (float)(int16_t)(w[0] & 0xffff) * s;
    lo.y = (float)(int16_t)(w[0] >> 16) * s;
    lo.z = (float)(int16_t)(w[1] & 0xffff) * s;
    lo.w = (float)(int16_t)(w[1] >> 16) * s;
    hi.x = (float)(int16_t)(w[2] & 0xffff) * s;
    hi.y = (float)(int16_t)(w[2] >> 16) * s;
    hi.z = (float)(int16_t)(w[3] & 0xffff) * s;
    hi.w = (float)(int16_t)(w[3] >> 16) * s;
    reinterpret_cast<float4*>(y)[2 * i] = lo;
    reinterpret_cast<float4*>(y)[2 * i + 1] = hi;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const int64_t k = (n8 << 3) + threadIdx.x;
    y[k] = (float)x[k] * s;
  }
}

int launch_pcm16_to_f32(const int16_t* x, int64_t n, float* y, hipStream_t st) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 15)) {
    set_error("pcm16_to_f32: buffers must be 16-byte aligned");
    return -2;
  }
  const int64_t n8 = n >> 3;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n8 + 255) / 256, 256 * 16));
  hipLaunchKernelGGL(pcm16_to_f32_kernel, dim3(grid), dim3(256), 0, st, x, n, y);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

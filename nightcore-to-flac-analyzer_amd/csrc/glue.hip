// glue.hip — the small data-dependent steps between the heavy kernels, kept on
// the device so a whole batch runs stream-ordered with no host round trip:
//
//   energy_gate_kernel    io.energy_gate (io.py:115-126): keep windows with
//                         energy_db >= max(file) + threshold_db
//   collect_valid_kernel  consensus._valid (consensus.py:236-240) applied to the
//                         per-window tempo lists: ordered compaction of windows
//                         that are active, have >= 4 beats (tempo.py:54-55) and a
//                         finite positive tempo
//   pitch_hz_kernel       pitch.py:95 + 161-164: shift = lag / 3.0 (the quirk),
//                         nc_hz = 440 * 2^(shift/12), src_hz = 440
//   xcorr_peak_kernel     pitch._cyclic_xcorr_peak (pitch.py:67-85) for vectors of any
//                         length n (the 12-bin chroma_lag_kernel is the batch path)
#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

__global__ void energy_gate_kernel(const double* energy, const int* w0, const int* w1, int n_groups, double gate_db,
                                   uint8_t* active) {
  const int g = blockIdx.x;
  if (g >= n_groups) return;
  __shared__ double mx;
  if (threadIdx.x == 0) {
    double m = -INFINITY;
    for (int w = w0[g]; w < w1[g]; ++w) m = fmax(m, energy[w]);
    mx = m;
  }
  __syncthreads();
  for (int w = w0[g] + threadIdx.x; w < w1[g]; w += blockDim.x) active[w] = energy[w] >= mx + gate_db;
}

__global__ void collect_valid_kernel(const double* bpm, const int* nbeats, const uint8_t* active, const int* w0,
                                     const int* w1, int n_groups, int min_beats, double* out_values, int* out_n) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  int n = 0;
  for (int w = w0[g]; w < w1[g]; ++w) {
    const double v = bpm[w];
    if ((active == nullptr || active[w]) && nbeats[w] >= min_beats && isfinite(v) && v > 0.0)
      out_values[w0[g] + n++] = v;
  }
  out_n[g] = n;
}

__global__ void pitch_hz_kernel(const int* lags, int n, double* shift_out, double* nc_hz, double* src_hz) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double st = (double)lags[i] / 3.0;
  shift_out[i] = st;
  nc_hz[i] = 440.0 * pow(2.0, st / 12.0);
  src_hz[i] = 440.0;
}

// io._rms_db (io.py:38-40) for windows given by absolute offsets: 20 log10(max(rms_f64, 1e-10))
__global__ __launch_bounds__(256) void window_energy_kernel(const float* sig, const int64_t* off, int win_len,
                                                            double* out) {
  __shared__ BlockScratch<256> bs;
  const float* x = sig + off[blockIdx.x];
  double e = 0.0;
  for (int i = threadIdx.x; i < win_len; i += 256) {
    const double v = (double)x[i];
    e = fma(v, v, e);
  }
  e = block_sum<256>(e, bs);
  if (threadIdx.x == 0) out[blockIdx.x] = 20.0 * log10(fmax(sqrt(e / (double)win_len), 1e-10));
}

int launch_window_energy(const float* sig, const int64_t* off, int n, int win_len, double* out, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(window_energy_kernel, dim3(n), dim3(256), 0, st, sig, off, win_len, out);
  NC_HIP(hipGetLastError());
  return 0;
}

// profile mode 5 (MarkSpan, nc_prof.cpp): the wall clock when the stream reaches this launch,
// into the span slot's first line (start: min, end: max), as span_record does for a kernel
__global__ void span_mark_kernel(unsigned long long* sp, int end) {
  const unsigned long long t = wall_clock64();
  if (end) atomicMax(sp + 1, t);
  else atomicMin(sp, t);
}

int launch_span_mark(unsigned long long* span, int end, hipStream_t st) {
  hipLaunchKernelGGL(span_mark_kernel, dim3(1), dim3(1), 0, st, span, end);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_energy_gate(const double* energy, const int* w0, const int* w1, int n_groups, double gate_db,
                       uint8_t* active, hipStream_t st) {
  if (n_groups <= 0) return 0;
  hipLaunchKernelGGL(energy_gate_kernel, dim3(n_groups), dim3(64), 0, st, energy, w0, w1, n_groups, gate_db, active);
  NC_HIP(hipGetLastError());
  return 0;
}

int launch_collect_valid(const double* bpm, const int* nbeats, const uint8_t* active, const int* w0, const int* w1,
                         int n_groups, int min_beats, double* out_values, int* out_n, hipStream_t st) {
  if (n_groups <= 0) return 0;
  hipLaunchKernelGGL(collect_valid_kernel, dim3((n_groups + 63) / 64), dim3(64), 0, st, bpm, nbeats, active, w0, w1,
                     n_groups, min_beats, out_values, out_n);
  NC_HIP(hipGetLastError());
  return 0;
}

int launch_pitch_hz(const int* lags, int n, double* shift_out, double* nc_hz, double* src_hz, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(pitch_hz_kernel, dim3((n + 63) / 64), dim3(64), 0, st, lags, n, shift_out, nc_hz, src_hz);
  NC_HIP(hipGetLastError());
  return 0;
}

// pitch._cyclic_xcorr_peak for any n (pitch.py:67-85): xcorr[k] = sum_j a[j] b[(j + k) % n] as
// an f32 fma chain in j order (the 12-bin chroma_lag_kernel's arithmetic), first argmax with
// numpy's NaN rule (the first NaN wins), wrapped to lag - n when lag > n / 2.  One workgroup
// per pair; each thread scans lags k = tid, tid + 256, ..., then a (value, k) tree in LDS.
__device__ __forceinline__ bool xc_better(float v, int k, float bv, int bk) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || k < bk);
  return v > bv || (v == bv && k < bk);
}

__global__ __launch_bounds__(256) void xcorr_peak_kernel(const float* a, const float* b, int n, int* lag_out) {
  __shared__ float sv[256];
  __shared__ int sk[256];
  const float* x = a + (size_t)blockIdx.x * n;
  const float* y = b + (size_t)blockIdx.x * n;
  float bv = 0.0f;
  int bk = 0x7fffffff;
  for (int k = threadIdx.x; k < n; k += 256) {
    float d = 0.0f;
    int i = k;
    for (int j = 0; j < n; ++j) {
      d = fmaf(x[j], y[i], d);
      if (++i == n) i = 0;
    }
    if (bk == 0x7fffffff || xc_better(d, k, bv, bk)) {
      bv = d;
      bk = k;
    }
  }
  sv[threadIdx.x] = bv;
  sk[threadIdx.x] = bk;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const float v2 = sv[threadIdx.x + s];
      const int k2 = sk[threadIdx.x + s];
      if (k2 != 0x7fffffff && (sk[threadIdx.x] == 0x7fffffff || xc_better(v2, k2, sv[threadIdx.x], sk[threadIdx.x]))) {
        sv[threadIdx.x] = v2;
        sk[threadIdx.x] = k2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int lag = sk[0];
    lag_out[blockIdx.x] = lag > n / 2 ? lag - n : lag;
  }
}

int launch_xcorr_peak(const float* a, const float* b, int n, int n_pairs, int* lag_out, hipStream_t st) {
  if (n_pairs <= 0) return 0;
  if (n <= 0) {
    set_error("xcorr_peak: n must be positive (np.argmax of an empty sequence raises)");
    return -2;
  }
  hipLaunchKernelGGL(xcorr_peak_kernel, dim3(n_pairs), dim3(256), 0, st, a, b, n, lag_out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

// xcorr.hip — K13: windowed normalised waveform cross-correlation speed
// estimate, replacing the search loop of xcorr.estimate_speed_xcorr
// (xcorr.py:109-160).  oracle: refglue.estimate_speed_xcorr_arrays.
//
// The host plans the integer geometry exactly as the reference does (edge trim,
// linspace(0, len_a - win, n_windows).astype(int) positions, range(lo, hi,
// stride) candidates) and hands the engine a flat list of (a_offset, b_offset)
// dot products of `win` samples: one workgroup per dot product (f64
// accumulation of f32 samples, wave shuffles + LDS for the block sum).
// A finalize kernel (one thread per job) applies the reference's decisions in
// order: rms gate, norm gates, strict-'>' first maximum, best > 0, >= 3
// correspondences, least-squares slope (np.polyfit deg 1) and median quality.
#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

__global__ __launch_bounds__(256) void xcorr_dot_kernel(const float* sig, const int64_t* ia, const int64_t* ib,
                                                        int win, double* dot_out, double* sqb_out) {
  __shared__ BlockScratch<256> bs;
  const int it = blockIdx.x;
  const float* a = sig + ia[it];
  const float* b = sig + ib[it];
  double d = 0.0, q = 0.0;
  for (int i = threadIdx.x; i < win; i += 256) {
    const double x = (double)a[i], y = (double)b[i];
    d = fma(x, y, d);
    q = fma(y, y, q);
  }
  d = block_sum<256>(d, bs);
  q = block_sum<256>(q, bs);
  if (threadIdx.x == 0) {
    dot_out[it] = d;
    sqb_out[it] = q;
  }
}

// per job: windows [w0[j], w1[j]); window w: self item sw[w] (dot = sum a^2),
// candidate items [c0[w], c1[w]) with b positions pbv[item]; pa[w]; exp_pb[w].
__global__ void xcorr_finalize_kernel(const double* dot, const double* sqb, const int* w0, const int* w1,
                                      const int* sw, const int* c0, const int* c1, const int64_t* pa,
                                      const int64_t* pbv, const int64_t* exp_pb, int win, int n_jobs,
                                      double* ratio_out, double* quality_out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  double xa[64], xb[64], ql[64];
  int n = 0;
  for (int w = w0[j]; w < w1[j] && n < 64; ++w) {
    const double sa = dot[sw[w]];
    if (sqrt(sa / (double)win) < 1e-3) continue;       // xcorr.py:117-118 rms gate
    const double na = sqrt(sa);
    if (na < 1e-10) continue;                          // xcorr.py:127-129
    double best = -1.0;
    int64_t best_pb = exp_pb[w];
    for (int it = c0[w]; it < c1[w]; ++it) {
      const double nb = sqrt(sqb[it]);
      if (nb < 1e-10) continue;
      const double c = dot[it] / (na * nb);
      if (c > best) {                                   // strict '>' keeps the first maximum
        best = c;
        best_pb = pbv[it];
      }
    }
    if (best > 0) {
      xa[n] = (double)pa[w];
      xb[n] = (double)best_pb;
      ql[n] = best;
      ++n;
    }
  }
  if (n < 3) {
    ratio_out[j] = 1.0;
    quality_out[j] = 0.0;
    return;
  }
  double ma = 0.0, mb = 0.0;
  for (int i = 0; i < n; ++i) {
    ma += xa[i];
    mb += xb[i];
  }
  ma /= n;
  mb /= n;
  double sab = 0.0, saa = 0.0;
  for (int i = 0; i < n; ++i) {
    sab += (xa[i] - ma) * (xb[i] - mb);
    saa += (xa[i] - ma) * (xa[i] - ma);
  }
  ratio_out[j] = sab / saa;
  // median quality (insertion sort, n <= 64)
  for (int i = 1; i < n; ++i) {
    const double v = ql[i];
    int k = i - 1;
    while (k >= 0 && ql[k] > v) {
      ql[k + 1] = ql[k];
      --k;
    }
    ql[k + 1] = v;
  }
  quality_out[j] = (n & 1) ? ql[n / 2] : (ql[n / 2 - 1] + ql[n / 2]) / 2.0;
}

int launch_xcorr(const float* sig, const int64_t* ia, const int64_t* ib, int n_items, int win, double* dot,
                 double* sqb, const int* w0, const int* w1, const int* sw, const int* c0, const int* c1,
                 const int64_t* pa, const int64_t* pbv, const int64_t* exp_pb, int n_jobs, double* ratio_out,
                 double* quality_out, hipStream_t st) {
  if (n_items > 0)
    hipLaunchKernelGGL(xcorr_dot_kernel, dim3(n_items), dim3(256), 0, st, sig, ia, ib, win, dot, sqb);
  if (n_jobs > 0)
    hipLaunchKernelGGL(xcorr_finalize_kernel, dim3((n_jobs + 63) / 64), dim3(64), 0, st, dot, sqb, w0, w1, sw,
                       c0, c1, pa, pbv, exp_pb, win, n_jobs, ratio_out, quality_out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

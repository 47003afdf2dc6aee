// nc_decim.h — the 2:1 half-band decimator shared by the CQT octave chain (cqt.hip,
// librosa's resample(scale=True) inside cqt: x sqrt(2)) and the auto-align envelopes
// (align.hip, librosa.resample(scale=False) in xcorr.find_content_offset).  It replaces
// soxr_hq, which is absent (oracle/ncref.py halfband_taps / decimate2 / resample_half).
#pragma once
#include "nc_engine.h"

namespace nc {

// out[m] = s * sum_{j=0}^{2K} h[j] in[2m - (j - K)]  (zero outside), in the oracle's order
// (ascending j: oracle/ncref.py decimate2) with one fused multiply-add per tap, s = sqrt(2)
// or 1.  Acc = double (the auto-align envelopes: < 1e-16 relative to the oracle's separately
// rounded products) or float (the CQT octave chain: ~1e-7 relative per level, 2x the
// throughput and half the LDS of f64; the CQT's own f32 FFTs sit at the same level and the
// chroma parity bar is 2e-5, tests/test_gpu_chroma.py).  One workgroup of 256 threads per
// DEC_OUT outputs; the 2 DEC_OUT + 2K input tile is staged in LDS and the taps are
// wave-uniform (scalar loads); the zero taps of the half-band (even j - K != 0) are skipped
// at compile time.
constexpr int DEC_OUT = 1024;  // outputs per workgroup: 4 consecutive per thread

__device__ __forceinline__ int dec_pad(int e) { return e + (e >> 3); }  // softens stride-4 bank reuse

template <bool SQRT2, typename Acc = double>
__device__ __forceinline__ void halfband_tile(const float* in, int64_t Lin, float* out, int64_t Lout, int64_t m0,
                                              const double* __restrict__ taps) {
  constexpr int K = kHalfbandK;      // 23: taps j - K odd (24 of them) plus the centre
  constexpr int H = (K + 1) / 2;      // 12
  constexpr int W = 4 + 2 * H - 1;    // odd-phase window of 4 consecutive outputs: 27 values
  // in[2m - n] with n = j - K: the centre reads the even phase at m, odd n read the odd
  // phase at m + c, c = (-n - 1) / 2 in [-H, H - 1].  Both phases are staged in LDS as Acc;
  // one float2 load fetches one even and one odd sample (coalesced, every input read once).
  __shared__ Acc te[DEC_OUT + DEC_OUT / 8];
  __shared__ Acc to[DEC_OUT + 2 * H + (DEC_OUT + 2 * H) / 8 + 1];
  // pair p = (in[2p], in[2p + 1]) for p in [m0 - H, m0 + DEC_OUT + H); to[u] = odd phase at m0 - H + u
  const bool vec = ((reinterpret_cast<uintptr_t>(in) & 7) == 0);
  for (int u = threadIdx.x; u < DEC_OUT + 2 * H; u += 256) {
    const int64_t pidx = m0 - H + u;
    const int64_t i = 2 * pidx;
    Acc e = 0, o = 0;
    if (vec && i >= 0 && i + 1 < Lin) {
      const float2 v = reinterpret_cast<const float2*>(in)[pidx];
      e = (Acc)v.x;
      o = (Acc)v.y;
    } else {
      if (i >= 0 && i < Lin) e = (Acc)in[i];
      if (i + 1 >= 0 && i + 1 < Lin) o = (Acc)in[i + 1];
    }
    if (u >= H && u < H + DEC_OUT) te[dec_pad(u - H)] = e;
    to[dec_pad(u)] = o;
  }
  __syncthreads();
  const int l0 = 4 * threadIdx.x;
  Acc xo[W], xe[4];
#pragma unroll
  for (int i = 0; i < W; ++i) xo[i] = to[dec_pad(l0 + i)];
#pragma unroll
  for (int q = 0; q < 4; ++q) xe[q] = te[dec_pad(l0 + q)];
  Acc acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j <= 2 * K; ++j) {  // the oracle's order (ascending j), one FMA per tap
    const int n = j - K;
    if (n != 0 && !(n & 1)) continue;
    const Acc h = (Acc)taps[j];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = fma(h, n == 0 ? xe[q] : xo[q + H + (-n - 1) / 2], acc[q]);
  }
  float r[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = SQRT2 ? (float)((double)acc[q] * 1.4142135623730951) : (float)acc[q];
  const int64_t m = m0 + l0;
  if (m + 3 < Lout && ((reinterpret_cast<uintptr_t>(out + m) & 15) == 0)) {
    *reinterpret_cast<float4*>(out + m) = make_float4(r[0], r[1], r[2], r[3]);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (m + q < Lout) out[m + q] = r[q];
  }
}

}  // namespace nc

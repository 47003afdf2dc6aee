// nc_tgcorr.h — the frame-averaged tempogram as six lag correlations.
//
// librosa.feature.tempogram (beat_track's tempo estimate, tempo.py:45/63) autocorrelates
// every Hann-windowed frame of the ramp-padded onset envelope x, normalises each frame by
// ac_t[0] and averages over the T frames (oracle/ncref.py tempogram_mean):
//   T tg[k] = sum_t r_t sum_{j < N-k} w[j] w[j+k] x[t+j] x[t+j+k],   r_t = 1 / ac_t[0].
// Substituting u = t + j,
//   T tg[k] = sum_u x[u] x[u+k] sum_{t = lo(u+k)}^{hi(u)} r_t G_k(u - t),
//   hi(u) = min(T-1, u),  lo(v) = max(0, v - N + 1),  G_k(j) = w[j] w[j+k],
// and with theta = 2 pi / N, (c, s) = (cos, sin)(theta k), the periodic Hann window gives
//   G_k(j) = A + B cos(theta j) + C sin(theta j) + D cos(2 theta j) + E sin(2 theta j),
//   A = 1/4 + c/8,  B = -1/4 - c/4,  C = s/4,  D = c/8,  E = -s/8.
// Expanding cos(theta (u - t)) etc., the inner sum is a combination of the five prefix
// sums Q_m(n) = sum_{t<n} r_t f_m(t), f = (1, cos theta t, sin theta t, cos 2 theta t,
// sin 2 theta t), taken at hi(u)+1 (a term that depends on u only) minus at lo(u+k) (a
// term that depends on v = u + k only).  Collecting the k-dependence into
// phi(k) = (1, c, s), every lag needs only
//   T tg[k] = sum_{i<3} phi_i(k) (sum_u a_i[u] x[u+k] - sum_v b_i[v] x[v-k]),
//   a_i[u] = x[u] g_i(P(hi(u)+1), u),  b_i[v] = x[v] g_i(P(lo(v)), v) (third one negated),
//   P0 = Q0,  P1 = cu Qc1 + su Qs1,  P2 = su Qc1 - cu Qs1,  P3 = c2u Qc2 + s2u Qs2,
//   P4 = s2u Qc2 - c2u Qs2,  g = ((P0 - P1)/4, P0/8 - P1/4 + P3/8, P2/4 - P4/8),
// six correlations over u in [0, T + N), x zero outside its T + 2 (N/2) samples.  That is
// 6 FMAs per (lag, sample) against ~28 flops per (lag, frame) for sliding sums, with no
// loop-carried recurrence, so the lags x samples grid is spread over the whole workgroup;
// the conditioning is no worse than the recurrences' (a prefix sum is never differenced
// against a far-away one inside the same product), see tests/test_oracle_known_answers.py.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace nc {

// consecutive lags per thread (odd: 6-dword lane stride, no LDS bank conflicts; 5 spills)
constexpr int TGC_LB = 3;

__host__ __device__ inline int tgc_extent(int T, int N) { return T + N; }       // u range
__host__ __device__ inline int tgc_pad(int N) { return N + TGC_LB + 1; }        // zeros either side of x
__host__ __device__ inline int tgc_blocks(int N) { return (N + TGC_LB - 1) / TGC_LB; }
__host__ __device__ inline int tgc_segments(int N, int nthreads) {
  const int s = nthreads / tgc_blocks(N);
  return s > 0 ? s : 1;
}

// Q_m(n), n = 0..T, of r_t f_m(t) into q[m (T + 1) + n]; cs[2 j] / cs[2 j + 1] = cos / sin(theta j).
// Waves 0..4 scan one array each: 64 contiguous runs, then a fixed-order wave scan of the runs.
__device__ __forceinline__ void tgc_prefix(const double* rinv, const double* cs, int T, int N, double* q, int tid,
                                           int nthreads) {
  const int wave = tid >> 6, lane = tid & 63;
  if (wave >= 5 || nthreads < 320) {
    if (nthreads < 320 && tid == 0) {  // small blocks: serial scans (not used by the kernels here)
      for (int m = 0; m < 5; ++m) {
        double acc = 0.0;
        q[m * (T + 1)] = 0.0;
        for (int t = 0; t < T; ++t) {
          const int j = (m <= 2 ? t : 2 * t) % N;
          acc += m == 0 ? rinv[t] : rinv[t] * cs[2 * j + ((m & 1) ? 0 : 1)];
          q[m * (T + 1) + t + 1] = acc;
        }
      }
    }
    return;
  }
  const int m = wave;
  auto f = [&](int t) -> double {
    if (m == 0) return rinv[t];
    const int j = (m <= 2 ? t : 2 * t) % N;
    return rinv[t] * cs[2 * j + ((m & 1) ? 0 : 1)];
  };
  const int C = (T + 63) / 64;
  const int t0 = min(T, lane * C), t1 = min(T, t0 + C);
  double s = 0.0;
  for (int t = t0; t < t1; ++t) s += f(t);
  double incl = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double v = __shfl_up(incl, off);
    if (lane >= off) incl += v;
  }
  double run = __shfl_up(incl, 1);
  if (lane == 0) run = 0.0;
  double* qm = q + m * (T + 1);
  if (lane == 0) qm[0] = 0.0;
  for (int t = t0; t < t1; ++t) {
    run += f(t);
    qm[t + 1] = run;
  }
}

// The six sequences: seq[i U + u] = a_i[u] (i < 3), seq[(3 + i) U + u] = b_i[u].
__device__ __forceinline__ void tgc_sequences(const double* x, const double* q, const double* cs, int T, int N,
                                              int U, double* seq, int tid, int nthreads) {
  for (int u = tid; u < U; u += nthreads) {
    const double xv = x[u];
    const int i1 = u % N, i2 = (2 * u) % N;
    const double cu = cs[2 * i1], su = cs[2 * i1 + 1], c2u = cs[2 * i2], s2u = cs[2 * i2 + 1];
    auto g = [&](int at, double& g0, double& g1, double& g2) {
      const double P0 = q[at], Qc1 = q[(T + 1) + at], Qs1 = q[2 * (T + 1) + at];
      const double Qc2 = q[3 * (T + 1) + at], Qs2 = q[4 * (T + 1) + at];
      const double P1 = cu * Qc1 + su * Qs1, P2 = su * Qc1 - cu * Qs1;
      const double P3 = c2u * Qc2 + s2u * Qs2, P4 = s2u * Qc2 - c2u * Qs2;
      g0 = 0.25 * (P0 - P1);
      g1 = 0.125 * P0 - 0.25 * P1 + 0.125 * P3;
      g2 = 0.25 * P2 - 0.125 * P4;
    };
    double a0, a1, a2, b0, b1, b2;
    g(min(T - 1, u) + 1, a0, a1, a2);
    g(max(0, u - N + 1), b0, b1, b2);
    seq[u] = xv * a0;
    seq[U + u] = xv * a1;
    seq[2 * U + u] = xv * a2;
    seq[3 * U + u] = xv * b0;
    seq[4 * U + u] = xv * b1;
    seq[5 * U + u] = -(xv * b2);
  }
}

template <int I, int N_, class F>
__device__ __forceinline__ void tgc_static_for_impl(F&& f) {
  if constexpr (I < N_) {
    f(std::integral_constant<int, I>{});
    tgc_static_for_impl<I + 1, N_>(f);
  }
}
template <int N_, class F>
__device__ __forceinline__ void tgc_static_for(F&& f) { tgc_static_for_impl<0, N_>(f); }

// part[s stride + k] = the lag-k correlation combination over the s-th u segment;
// stride = tgc_blocks(N) TGC_LB, segments = tgc_segments(N, nthreads).  Each thread
// holds TGC_LB consecutive lags: x[u + k] and x[u - k] slide through registers, so a
// sample costs 6 broadcast sequence reads + 2 x reads for 6 TGC_LB FMAs.
__device__ __forceinline__ void tgc_correlate(const double* x, const double* seq, int N, int U, double* part, int tid,
                                              int nthreads) {
  constexpr int LB = TGC_LB;
  const int nblk = tgc_blocks(N), nseg = tgc_segments(N, nthreads), stride = nblk * LB;
  for (int task = tid; task < nblk * nseg; task += nthreads) {
    const int blk = task % nblk, s = task / nblk, k0 = blk * LB;
    const int ua = (int)((int64_t)U * s / nseg), ub = (int)((int64_t)U * (s + 1) / nseg);
    double h0[LB], h1[LB], h2[LB], z0[LB], z1[LB], z2[LB], xp[LB], xm[LB];
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      h0[q] = h1[q] = h2[q] = z0[q] = z1[q] = z2[q] = 0.0;
      xp[q] = xm[q] = 0.0;
    }
#pragma unroll
    for (int q = 0; q < LB - 1; ++q) {
      xp[q] = x[ua + k0 + q];           // x[u + k0 + q]
      xm[q] = x[ua - k0 - LB + 1 + q];  // x[u - k0 - (LB - 1) + q]
    }
    // one step at sample u, window rotation r: logical slot q of xp / xm lives in register
    // (q + r) % LB, so a full unrolled group of LB steps needs no register moves
    auto step = [&](int u, auto rot) {
      constexpr int r = decltype(rot)::value;
      xp[(r + LB - 1) % LB] = x[u + k0 + LB - 1];
      xm[(r + LB - 1) % LB] = x[u - k0];
      const double a0 = seq[u], a1 = seq[U + u], a2 = seq[2 * U + u];
      const double b0 = seq[3 * U + u], b1 = seq[4 * U + u], b2 = seq[5 * U + u];
#pragma unroll
      for (int q = 0; q < LB; ++q) {
        const double vp = xp[(r + q) % LB], vm = xm[(r + LB - 1 - q) % LB];
        h0[q] = fma(a0, vp, h0[q]);
        h1[q] = fma(a1, vp, h1[q]);
        h2[q] = fma(a2, vp, h2[q]);
        z0[q] = fma(b0, vm, z0[q]);
        z1[q] = fma(b1, vm, z1[q]);
        z2[q] = fma(b2, vm, z2[q]);
      }
    };
    int u = ua;
#pragma unroll 1
    for (; u + LB <= ub; u += LB) tgc_static_for<LB>([&](auto rot) { step(u + decltype(rot)::value, rot); });
    tgc_static_for<LB>([&](auto rot) {
      if (u + decltype(rot)::value < ub) step(u + decltype(rot)::value, rot);
    });
    const double inv_half = 2.0 / (double)N;
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int k = k0 + q;
      if (k < N) {
        double sk, ck;
        sincospi((double)k * inv_half, &sk, &ck);
        part[s * stride + k] = (h0[q] - z0[q]) + ck * (h1[q] - z1[q]) + sk * (h2[q] - z2[q]);
      }
    }
  }
}

}  // namespace nc

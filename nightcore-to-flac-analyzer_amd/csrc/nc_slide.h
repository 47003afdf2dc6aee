// nc_slide.h — the tempogram autocorrelation as five sliding f64 sums.
//
// librosa.feature.tempogram (via beat_track's tempo estimate, tempo.py:45/63)
// autocorrelates every Hann-windowed frame of the ramp-padded onset envelope x:
//   ac_t[k] = sum_{j < N-k} w[j] w[j+k] x[t+j] x[t+j+k],   w = periodic Hann(N),
// normalises each frame by max_k |ac_t[k]| (= ac_t[0]) and averages over t
// (oracle/ncref.py tempogram_mean).  With theta = 2 pi / N the product of two
// shifted Hann windows is a trigonometric polynomial of degree 2 in j:
//   w[j] w[j+k] = A + B cos(theta j) + C sin(theta j) + D cos(2 theta j) + E sin(2 theta j)
//   A = 1/4 + c/8,  B = -1/4 - c/4,  C = s/4,  D = c/8,  E = -s/8,   (c, s) = (cos, sin)(theta k).
// With p_k[u] = x[u] x[u+k] and L = N - k this gives
//   ac_t[k] = A S0(t) + B Re Z1(t) + C Im Z1(t) + D Re Z2(t) + E Im Z2(t),
//   S0(t) = sum_{j<L} p_k[t+j],   Zm(t) = sum_{j<L} e^{i m theta j} p_k[t+j],
// and every sum slides one frame in O(1):
//   Zm(t+1) = e^{-i m theta} (Zm(t) - p_k[t] + e^{i m theta L} p_k[t+L]),  e^{i m theta L} = e^{-i m theta k}.
// All arithmetic is f64: about 28 flops per (lag, frame), against two 2N-point
// FFTs per frame, and agreement with librosa's f64 FFT autocorrelation at the
// 1e-15 level (tests/test_oracle_known_answers.py checks the identity).
#pragma once
#include <hip/hip_runtime.h>

namespace nc {

// sum_{t0 <= t < t1} ac_t[k] * rinv(t); x(i) returns the padded envelope (float),
// valid for t0 <= i < t1 - 1 + N + 1.
template <class XF, class RF>
__device__ __forceinline__ double slide_lag_sum(const XF& x, const RF& rinv, int N, int k, int t0, int t1) {
  const double inv_half = 2.0 / (double)N;  // theta / pi
  double s1, c1, sk, ck;
  sincospi(inv_half, &s1, &c1);
  sincospi((double)k * inv_half, &sk, &ck);
  const double c2 = fma(c1, c1, -s1 * s1), s2 = 2.0 * c1 * s1;
  const double ck2 = fma(ck, ck, -sk * sk), sk2 = 2.0 * ck * sk;
  const double A = 0.25 + 0.125 * ck, B = -0.25 - 0.25 * ck, C = 0.25 * sk, D = 0.125 * ck, E = -0.125 * sk;
  const int L = N - k;

  double S0 = 0.0, z1r = 0.0, z1i = 0.0, z2r = 0.0, z2i = 0.0;
  for (int j0 = 0; j0 < L; j0 += 64) {
    double es, ec;  // e^{i theta j}, re-seeded every 64 terms
    sincospi((double)j0 * inv_half, &es, &ec);
    const int je = min(L, j0 + 64);
    for (int j = j0; j < je; ++j) {
      const double p = (double)x(t0 + j) * (double)x(t0 + j + k);
      const double e2c = fma(ec, ec, -es * es), e2s = 2.0 * ec * es;
      S0 += p;
      z1r = fma(ec, p, z1r);
      z1i = fma(es, p, z1i);
      z2r = fma(e2c, p, z2r);
      z2i = fma(e2s, p, z2i);
      const double nc = fma(ec, c1, -es * s1), ns = fma(es, c1, ec * s1);
      ec = nc;
      es = ns;
    }
  }
  double acc = 0.0;
  for (int t = t0; t < t1; ++t) {
    const double ac = fma(E, z2i, fma(D, z2r, fma(C, z1i, fma(B, z1r, A * S0))));
    acc = fma(ac, rinv(t), acc);
    const double pt = (double)x(t) * (double)x(t + k);
    const double pl = (double)x(t + L) * (double)x(t + N);
    S0 = (S0 - pt) + pl;
    // (u) * e^{-i m theta}:  (a + ib)(c - is) = (ac + bs) + i(bc - as)
    const double u1r = fma(ck, pl, z1r - pt), u1i = fma(-sk, pl, z1i);
    z1r = fma(u1r, c1, u1i * s1);
    z1i = fma(u1i, c1, -u1r * s1);
    const double u2r = fma(ck2, pl, z2r - pt), u2i = fma(-sk2, pl, z2i);
    z2r = fma(u2r, c2, u2i * s2);
    z2i = fma(u2i, c2, -u2r * s2);
  }
  return acc;
}

// Normaliser of one frame: 1 / ac_t[0] (librosa util.normalize(norm=inf) with
// threshold tiny(f64): a frame whose max is below tiny is left as is).
__device__ __forceinline__ double tg_rinv(double ac0) { return ac0 < 2.2250738585072014e-308 ? 1.0 : 1.0 / ac0; }

}  // namespace nc

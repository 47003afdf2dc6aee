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
  // operands of frame t are loaded one frame ahead (software pipelining: the LDS latency
  // overlaps the previous frame's arithmetic); x must be readable up to t1 + N
  double xt = (double)x(t0), xk = (double)x(t0 + k), xl = (double)x(t0 + L), xn = (double)x(t0 + N);
  double r = rinv(t0);
  for (int t = t0; t < t1; ++t) {
    const int tn = t + 1 < t1 ? t + 1 : t;
    const double xt1 = (double)x(tn), xk1 = (double)x(tn + k), xl1 = (double)x(tn + L), xn1 = (double)x(tn + N);
    const double r1 = rinv(tn);
    const double ac = fma(E, z2i, fma(D, z2r, fma(C, z1i, fma(B, z1r, A * S0))));
    acc = fma(ac, r, acc);
    const double pt = xt * xk;
    const double pl = xl * xn;
    xt = xt1;
    xk = xk1;
    xl = xl1;
    xn = xn1;
    r = r1;
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

// Per-lag state of the sliding sums (see the header comment).
struct SlideLag {
  double A, B, C, D, E;      // w[j] w[j+k] expansion coefficients
  double ck, sk, ck2, sk2;   // e^{-i theta k}, e^{-2 i theta k} (= e^{i m theta L})
  double S0, z1r, z1i, z2r, z2i;
  int k, L;
};

template <class XF>
__device__ __forceinline__ void slide_init(SlideLag& s, const XF& x, int N, int k, int t0, double c1, double s1) {
  const double inv_half = 2.0 / (double)N;
  double sk, ck;
  sincospi((double)k * inv_half, &sk, &ck);
  s.k = k;
  s.L = N - k;
  s.ck = ck;
  s.sk = sk;
  s.ck2 = fma(ck, ck, -sk * sk);
  s.sk2 = 2.0 * ck * sk;
  s.A = 0.25 + 0.125 * ck;
  s.B = -0.25 - 0.25 * ck;
  s.C = 0.25 * sk;
  s.D = 0.125 * ck;
  s.E = -0.125 * sk;
  double S0 = 0.0, z1r = 0.0, z1i = 0.0, z2r = 0.0, z2i = 0.0;
  for (int j0 = 0; j0 < s.L; j0 += 64) {
    double es, ec;  // e^{i theta j}, re-seeded every 64 terms
    sincospi((double)j0 * inv_half, &es, &ec);
    const int je = min(s.L, j0 + 64);
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
  s.S0 = S0;
  s.z1r = z1r;
  s.z1i = z1i;
  s.z2r = z2r;
  s.z2i = z2i;
}

__device__ __forceinline__ double slide_ac(const SlideLag& s) {
  return fma(s.E, s.z2i, fma(s.D, s.z2r, fma(s.C, s.z1i, fma(s.B, s.z1r, s.A * s.S0))));
}

// advance one frame given p[t] and p[t + L]
__device__ __forceinline__ void slide_step(SlideLag& s, double pt, double pl, double c1, double s1, double c2,
                                           double s2) {
  s.S0 = (s.S0 - pt) + pl;
  const double u1r = fma(s.ck, pl, s.z1r - pt), u1i = fma(-s.sk, pl, s.z1i);
  s.z1r = fma(u1r, c1, u1i * s1);
  s.z1i = fma(u1i, c1, -u1r * s1);
  const double u2r = fma(s.ck2, pl, s.z2r - pt), u2i = fma(-s.sk2, pl, s.z2i);
  s.z2r = fma(u2r, c2, u2i * s2);
  s.z2i = fma(u2i, c2, -u2r * s2);
}

// Two lags at once (independent dependency chains interleaved; the x(t) and rinv(t)
// reads are shared).  Same arithmetic per lag as slide_lag_sum.
template <class XF, class RF>
__device__ __forceinline__ void slide_lag_sum2(const XF& x, const RF& rinv, int N, int ka, int kb, int t0, int t1,
                                               double& acc_a, double& acc_b) {
  double s1, c1;
  sincospi(2.0 / (double)N, &s1, &c1);
  const double c2 = fma(c1, c1, -s1 * s1), s2 = 2.0 * c1 * s1;
  SlideLag a, b;
  slide_init(a, x, N, ka, t0, c1, s1);
  slide_init(b, x, N, kb, t0, c1, s1);
  double ra = 0.0, rb = 0.0;
  // operands loaded one frame ahead (see slide_lag_sum)
  double xt = (double)x(t0), xn = (double)x(t0 + N), xka = (double)x(t0 + ka), xkb = (double)x(t0 + kb);
  double xla = (double)x(t0 + a.L), xlb = (double)x(t0 + b.L), r = rinv(t0);
  for (int t = t0; t < t1; ++t) {
    const int tn = t + 1 < t1 ? t + 1 : t;
    const double xt1 = (double)x(tn), xn1 = (double)x(tn + N), xka1 = (double)x(tn + ka), xkb1 = (double)x(tn + kb);
    const double xla1 = (double)x(tn + a.L), xlb1 = (double)x(tn + b.L), r1 = rinv(tn);
    ra = fma(slide_ac(a), r, ra);
    rb = fma(slide_ac(b), r, rb);
    slide_step(a, xt * xka, xla * xn, c1, s1, c2, s2);
    slide_step(b, xt * xkb, xlb * xn, c1, s1, c2, s2);
    xt = xt1;
    xn = xn1;
    xka = xka1;
    xkb = xkb1;
    xla = xla1;
    xlb = xlb1;
    r = r1;
  }
  acc_a = ra;
  acc_b = rb;
}

// Normaliser of one frame: 1 / ac_t[0] (librosa util.normalize(norm=inf) with
// threshold tiny(f64): a frame whose max is below tiny is left as is).
__device__ __forceinline__ double tg_rinv(double ac0) { return ac0 < 2.2250738585072014e-308 ? 1.0 : 1.0 / ac0; }

}  // namespace nc

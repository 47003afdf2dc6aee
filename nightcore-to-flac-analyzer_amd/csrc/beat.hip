// beat.hip — tempo estimate + dynamic-programming beat tracker (K6, K7, K8).
//
// Restates librosa 0.11 ``beat.beat_track(onset_envelope=..., start_bpm=...)``
// as called at tempo.py:45-50 (per 10 s window, hop 512) and tempo.py:159-164
// (full signal, hop 64), on top of the tempogram mean from window_stage /
// ibi.hip.  CPU restatement: oracle/ncref.py (tempo_from_tg, beat_local_score,
// beat_track_dp, last_beat, trim_beats).
//
// One workgroup per sequence.  The DP (cumscore[i] = ls[i] + max_d cum[i-d] -
// pen[d], d in [round(P/2), 2P]) is serial in i but every frame of a block of
// round(P/2) consecutive frames depends only on frames before the block, so a
// block is scored at once: threads split (frame, candidate chunk) pairs, the
// per-chunk winners meet in LDS and one thread per frame folds them — two
// barriers per block, no cross-lane shuffle chains.  Short sequences keep every
// array in LDS; long ones (hop-64 IBI pass) keep ls/cum/back in a global
// workspace and the last cumulative scores in an LDS ring.
//
// Decision arithmetic is float64 throughout (as librosa's numba kernels), with
// FMA contraction disabled where librosa adds separately rounded products.
#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

struct BeatArgs {
  const float* onset;
  const int64_t* off;
  const int* len;
  const double* tg;
  int acw;
  const double* start_bpm;
  const int* prior_idx;  // nullable: start = start_bpm[prior_idx[s]]
  const uint8_t* active; // nullable
  int sr, hop;
  double max_tempo;
  float tightness;
  int trim;
  double* bpm_out;
  int* lag_out;
  int* nbeats_out;
  double* margin_out;   // nullable
  int* beats_out;       // nullable (frames, at off[s])
  double* ws_ls;
  double* ws_cum;
  int* ws_back;
  uint8_t* ws_marks;
  int max_len;          // SMALL: LDS capacity in frames
  int tab_cap;          // doubles for the window / penalty table
  int ring_cap;         // !SMALL: LDS ring of the last ring_cap cumulative scores (power of 2)
  int phase;            // !SMALL: 0 one launch, 1 up to the normalised onset, 2 from the local score
  unsigned long long* span = nullptr;  // nc_profile execution span (nc_device.h)
};

__host__ __device__ __forceinline__ size_t al16(size_t n) { return (n + 15) & ~(size_t)15; }

// Workgroup barrier for LDS-only hand-offs: waits for this wave's LDS traffic but not for
// its outstanding global loads/stores (which __syncthreads' fence would drain every block).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifdef NC_BEAT_PROF
#define NC_BEAT_T(k) \
  do { __syncthreads(); if (threadIdx.x == 0) prof_t[k] = wall_clock64(); } while (0)
#define NC_BEAT_DUMP() \
  do { if (threadIdx.x == 0 && blockIdx.x == 0) printf("beatprof SMALL=%d N=%d P=%d: %ld %ld %ld %ld %ld %ld\n", (int)SMALL, N, Pi, \
       (long)(prof_t[1]-prof_t[0]), (long)(prof_t[2]-prof_t[1]), (long)(prof_t[3]-prof_t[2]), (long)(prof_t[4]-prof_t[3]), \
       (long)(prof_t[5]-prof_t[4]), (long)(prof_t[6]-prof_t[5])); } while (0)
#else
#define NC_BEAT_T(k) do {} while (0)
#define NC_BEAT_DUMP() do {} while (0)
#endif

// beat_track's local score: the onset envelope (normalised) convolved with a Gaussian
// window of 2P + 1 taps, exp(-0.5 ((k - P) 32 / P)^2), summed in ascending tap order
__device__ __forceinline__ double beat_window(int k, int Pi, double P) {
#pragma clang fp contract(off)
  const double v = ((double)(k - Pi) * 32.0) / P;
  return exp(-0.5 * (v * v));
}
__device__ __forceinline__ double beat_local_score(const float* onn, const double* tab, int i, int N, int Pi, int K) {
#pragma clang fp contract(off)
  const int klo = max(0, i + Pi - N + 1), khi = min(i + Pi, K - 1);
  const float* on = onn + i + Pi;
  double acc = 0.0;
  for (int k = klo; k <= khi; ++k) acc = acc + tab[k] * (double)on[-k];
  return acc;
}

// Long sequences, between phase 1 and phase 2 of tempo_beat_kernel<1024, false>: the local
// score of every frame, one frame per thread over the whole chip (a hop-64 60-min signal has
// ~1M frames x 2P + 1 taps, which one workgroup took ~27 ms over).
template <int NT>
__global__ __launch_bounds__(NT) void beat_localscore_kernel(BeatArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* ltab = reinterpret_cast<double*>(smem);
  const int s = blockIdx.y;
  if (a.active && !a.active[s]) return;
  const int N = a.len[s];
  if (N < 4 || (int64_t)blockIdx.x * NT >= N) return;
  const int64_t off = a.off[s];
  const int* meta = a.ws_back + off;
  if (meta[3] != 1) return;
  const int Pi = meta[0], K = 2 * Pi + 1;
  for (int k = threadIdx.x; k < K; k += NT) ltab[k] = beat_window(k, Pi, (double)Pi);
  __syncthreads();
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i < N) a.ws_ls[off + i] = beat_local_score(reinterpret_cast<const float*>(a.ws_cum + off), ltab, i, N, Pi, K);
}

constexpr int kBeatWin = 1024;  // long-sequence DP window (frames staged per global round trip)

template <int NT, bool SMALL>
__global__ __launch_bounds__(NT) void tempo_beat_kernel(BeatArgs a) {
#pragma clang fp contract(off)
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ BlockScratch<NT> bs;
  __shared__ int hist[256];
  __shared__ int sh_int[4];
  __shared__ double sel_med[2];
  __shared__ double dp_best[NT];
  __shared__ int dp_d[NT];
#ifdef NC_BEAT_PROF
  __shared__ long long prof_t[8];
#endif
  const int s = blockIdx.x;

  if (a.active && !a.active[s]) {
    if (threadIdx.x == 0) {
      a.bpm_out[s] = 0.0;
      a.lag_out[s] = 0;
      a.nbeats_out[s] = 0;
      if (a.margin_out) a.margin_out[s] = 0.0;
    }
    return;
  }
  const int N = a.len[s];
  const int64_t off = a.off[s];
  const float* onset = a.onset + off;
  const double* tg = a.tg + (size_t)s * a.acw;
  double* tab = reinterpret_cast<double*>(smem);
  char* p = smem + al16((size_t)a.tab_cap * sizeof(double));
  double *ls, *cum;
  int* back;
  uint8_t* marks;
  if (SMALL) {
    ls = reinterpret_cast<double*>(p);
    cum = ls + a.max_len;
    back = reinterpret_cast<int*>(cum + a.max_len);
    marks = reinterpret_cast<uint8_t*>(back + a.max_len);
  } else {
    ls = a.ws_ls + off;
    cum = a.ws_cum + off;
    back = a.ws_back + off;
    marks = a.ws_marks + off;
    if (a.phase == 1 && N >= 4 && threadIdx.x == 0) back[3] = 0;  // local-score meta: not ready
  }

  // ------------------------------------------------------------ any onset?
  int nz = 0;
  for (int i = threadIdx.x; i < N; i += NT) nz |= (onset[i] != 0.0f);
  nz = block_max_i<NT>(nz, bs);
  if (!nz) {  // beat_track: "if not onset_envelope.any(): return (0, [])"
    if (threadIdx.x == 0) {
      a.bpm_out[s] = 0.0;
      a.lag_out[s] = 0;
      a.nbeats_out[s] = 0;
      if (a.margin_out) a.margin_out[s] = 0.0;
    }
    return;
  }

  // ------------------------------------------------------------ tempo: prior-weighted argmax
  NC_BEAT_T(0);
  const double fs = (double)a.sr;
  const double start = a.prior_idx ? a.start_bpm[a.prior_idx[s]] : a.start_bpm[s];
  const double lstart = log2(start);
  // one pass keeps each thread's best and second best (numpy argmax order); the global
  // best L comes from the first, the runner-up (decision margin) from the second wherever
  // the thread's best is L itself
  double bv = -INFINITY, b2v = -INFINITY;
  int bi = 0x7fffffff, b2i = 0x7fffffff;
  for (int k = threadIdx.x; k < a.acw; k += NT) {
    double lp = -INFINITY;
    if (k > 0) {
      const double bpm = (60.0 * fs) / ((double)a.hop * (double)k);
      if (bpm < a.max_tempo) {
        const double d = (log2(bpm) - lstart) / 1.0;
        lp = -0.5 * (d * d);
      }
    }
    const double sc = log1p(1e6 * tg[k]) + lp;
    if (np_better(sc, k, bv, bi)) {
      b2v = bv;
      b2i = bi;
      bv = sc;
      bi = k;
    } else if (np_better(sc, k, b2v, b2i)) {
      b2v = sc;
      b2i = k;
    }
  }
  double sv = bv;
  int si = bi;
  block_argmax<NT>(bv, bi, bs);
  const int L = bi;
  if (si == L) {
    sv = b2v;
    si = b2i;
  }
  block_argmax<NT>(sv, si, bs);
  const double bpm = L > 0 ? (60.0 * fs) / ((double)a.hop * (double)L) : INFINITY;
  const double P = rint((fs / (double)a.hop) * 60.0 / bpm);
  if (threadIdx.x == 0) {
    a.bpm_out[s] = bpm;
    a.lag_out[s] = L;
    if (a.margin_out) a.margin_out[s] = bv - sv;
  }
  const int K = 2 * (int)P + 1;
  if (!(P >= 1.0) || K > a.tab_cap || (SMALL && N > a.max_len)) {
    if (threadIdx.x == 0) a.nbeats_out[s] = (P >= 1.0) ? -1 : 0;  // -1: capacity error
    return;
  }
  const int Pi = (int)P;

  // ------------------------------------------------------------ normalise + local score
  NC_BEAT_T(1);
  // Long sequences split this section over three launches (launch_tempo_beats): phase 1
  // stops after the normalised onset (meta in back[0..3]: P, -, -, ready), beat_localscore_kernel
  // fills ls[] across the chip, phase 2 starts from ls[].
  const bool split = !SMALL && a.phase != 0 && N >= 4;
  double lmax = -INFINITY;
  if (!split || a.phase == 1) {
    double sx = 0.0;
    for (int i = threadIdx.x; i < N; i += NT) sx += (double)onset[i];
    sx = block_sum<NT>(sx, bs);
    const float mean32 = (float)(sx / (double)N);
    double sq = 0.0;
    for (int i = threadIdx.x; i < N; i += NT) {
      const double d = (double)(onset[i] - mean32);
      sq += d * d;
    }
    sq = block_sum<NT>(sq, bs);
    const float std32 = (float)sqrt(sq / (double)(N - 1));
    const float norm = std32 + 1.17549435e-38f;

    // onset / norm once per frame (the same f32 quotient the per-tap form computed), kept in
    // cum's storage until the DP overwrites it
    float* onn = reinterpret_cast<float*>(cum);
    for (int i = threadIdx.x; i < N; i += NT) onn[i] = onset[i] / norm;
    if (split) {  // phase 1 ends here
      if (threadIdx.x == 0) {
        back[0] = Pi;
        back[3] = 1;
      }
      return;
    }
    for (int k = threadIdx.x; k < K; k += NT) tab[k] = beat_window(k, Pi, P);
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += NT) {
      const double acc = beat_local_score(onn, tab, i, N, Pi, K);
      ls[i] = acc;
      lmax = fmax(lmax, acc);
    }
  } else {
    for (int i = threadIdx.x; i < N; i += NT) lmax = fmax(lmax, ls[i]);
  }
  lmax = block_max<NT>(lmax, bs);
  const double thr = 0.01 * lmax;
  int first = N;
  for (int i = threadIdx.x; i < N; i += NT)
    if (!(ls[i] < thr)) first = min(first, i);
  const int i0 = block_min_i<NT>(first, bs);

  // ------------------------------------------------------------ DP
  NC_BEAT_T(2);
  const int dmin = (int)rint(P / 2.0);
  const int dmax = 2 * Pi;
  const double lP = log(P);
  const double tight = (double)a.tightness;
  __syncthreads();  // window table no longer needed
  for (int d = threadIdx.x; d <= dmax; d += NT) {
    const double t = log((double)d) - lP;
    tab[d] = tight * (t * t);
  }
  __syncthreads();
  // Frames [b0, b0 + B) with B <= dmin only read cum[] before b0, so a block of B frames is
  // scored at once: thread t takes frame t % B and the t / B-th of Gn consecutive chunks of
  // the candidate range [dmin, dmax]; per-chunk winners (ties: smaller d, as the ascending
  // scan) go to LDS and the B frame threads fold them in ascending chunk order.
  const int B = max(1, min(dmin, NT / 2));
  const int D = dmax - dmin + 1;
  // chunk length and fold length both ~sqrt(D): the scan and the fold are serial per thread
  const int Gn = max(1, min(min(NT / B, 64), (int)ceil(sqrt((double)D))));
  const int C = (D + Gn - 1) / Gn;
  // long sequences: the DP reads cum[i - d] for d in [dmin, dmax] only, so the last ring_cap
  // (>= dmax + B) scores are kept in an LDS ring instead of being re-read from L2 per candidate
  double* ring = SMALL ? cum : reinterpret_cast<double*>(smem + al16((size_t)a.tab_cap * sizeof(double)));
  const int RM = SMALL ? 0x7fffffff : a.ring_cap - 1;
  if (!SMALL && (dmax + B > a.ring_cap || kBeatWin > a.ring_cap)) {
    if (threadIdx.x == 0) a.nbeats_out[s] = -1;  // capacity error (cannot happen for P <= acw - 1)
    return;
  }
  const int f = threadIdx.x % B, g = threadIdx.x / B;
  const int dlo = dmin + g * C, dend = min(dmax + 1, dlo + C);
  // Long sequences run the DP in windows of FW frames (a multiple of B): ls of the window is
  // staged into LDS first, back[] collects in LDS, and cum / back go to global memory once
  // per window (from the ring, which still holds the window: FW <= ring_cap).  The blocks
  // themselves touch LDS only, so no block waits on a global round trip.  Short sequences
  // hold everything in LDS already: one window.
  const bool fthr = threadIdx.x < B;
  const int FW = SMALL ? N : max(B, (kBeatWin / B) * B);
  double* lsw = SMALL ? ls : ring + a.ring_cap;
  int* bkw = SMALL ? back : reinterpret_cast<int*>(lsw + kBeatWin);
  // Short sequences run the block DP on wave 0 alone, 8 lanes per frame: blocks of
  // Bq = min(dmin, 8) frames, lane (frame lane >> 3, chunk lane & 7) scans its eighth of the
  // candidate range [dmin, dmax] in ascending d (loads in batches of 8), the 8 chunk winners
  // of a frame meet by DPP (quad swaps, half-row mirror: no LDS round trip), and the chunk-0
  // lane writes cum / back.  The next block reads those scores through the wave's own
  // in-order LDS traffic, so no barrier or wait separates blocks.  Same candidates and the
  // same tie rule (largest score, then smallest d): bit-identical scores and back-pointers.
  const bool wave_dp = SMALL;
  if (wave_dp && threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int Bq = max(1, min(dmin, 8));
    const int Cw = (D + 7) / 8;
    const int fr = lane >> 3, gw = lane & 7;
    const int dlo_w = dmin + gw * Cw, dend_w = min(dmax + 1, dlo_w + Cw);
    auto take = [](double& best, int& bd, double v, int d) {
      if (v > best || (v == best && d < bd)) {
        best = v;
        bd = d;
      }
    };
    auto dpp_pair = [&](auto ctrl, double& best, int& bd) {
      constexpr int Cc = decltype(ctrl)::value;
      const long long bits = __double_as_longlong(best);
      const int lo = dpp_i<Cc>((int)(unsigned)bits, 0), hi = dpp_i<Cc>((int)(unsigned)(bits >> 32), 0);
      const double v = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
      take(best, bd, v, dpp_i<Cc>(bd, 0));
    };
    for (int b0 = 0; b0 < N; b0 += Bq) {
      const int i = b0 + fr;
      const bool valid = fr < Bq && i < N;
      double best = -INFINITY;
      int bd = 0x7fffffff;
      if (valid) {
        const int dh = min(dend_w, i + 1);
        for (int d0 = dlo_w; d0 < dh; d0 += 8) {
          double sc[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int d = min(d0 + u, dh - 1);  // past the range: a valid slot, masked below
            const double v = cum[i - d] - tab[d];
            sc[u] = d0 + u < dh ? v : -INFINITY;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (sc[u] > best) {
              best = sc[u];
              bd = d0 + u;
            }
        }
      }
      // all 64 lanes take part in the exchanges; the patterns stay inside a frame's 8 lanes
      dpp_pair(std::integral_constant<int, 0xB1>{}, best, bd);   // quad_perm [1,0,3,2]
      dpp_pair(std::integral_constant<int, 0x4E>{}, best, bd);   // quad_perm [2,3,0,1]
      dpp_pair(std::integral_constant<int, 0x141>{}, best, bd);  // row_half_mirror: the other quad
      if (valid && gw == 0) {
        const bool found = (i >= dmin) && (best > -INFINITY);
        cum[i] = found ? ls[i] + best : ls[i];
        back[i] = (i < i0 || !found) ? -1 : i - bd;
      }
      asm volatile("" ::: "memory");  // LDS traffic of one wave is in order; keep the compiler's too
    }
  }
  for (int w0 = 0; w0 < (wave_dp ? 0 : N); w0 += FW) {
    const int w1 = min(N, w0 + FW);
    if (!SMALL) {
      for (int q = threadIdx.x; q < w1 - w0; q += NT) lsw[q] = ls[w0 + q];
      __syncthreads();
    }
    for (int b0 = w0; b0 < w1; b0 += B) {
      const int i = b0 + f;
      const bool own = fthr && i < w1;
      const double lsi = own ? lsw[i - w0] : 0.0;
      if (g < Gn) {
        double best = -INFINITY;
        int bd = 0x7fffffff;
        if (i < w1) {
          const int dh = min(dend, i + 1);
          int d = dlo;
          for (; d + 3 < dh; d += 4) {
            double sc[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) sc[u] = ring[(i - d - u) & RM] - tab[d + u];
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (sc[u] > best) {
                best = sc[u];
                bd = d + u;
              }
          }
          for (; d < dh; ++d) {
            const double sc = ring[(i - d) & RM] - tab[d];
            if (sc > best) {
              best = sc;
              bd = d;
            }
          }
        }
        dp_best[threadIdx.x] = best;
        dp_d[threadIdx.x] = bd;
      }
      lds_barrier();
      if (own) {
        double best = -INFINITY;
        int bd = 0x7fffffff;
#pragma unroll 4
        for (int q = 0; q < Gn; ++q) {
          const double v = dp_best[q * B + f];
          const int d = dp_d[q * B + f];
          if (v > best || (v == best && d < bd)) {
            best = v;
            bd = d;
          }
        }
        const bool found = (i >= dmin) && (best > -INFINITY);
        const double v = found ? lsi + best : lsi;
        ring[i & RM] = v;  // = cum[i] for short sequences
        bkw[i - w0] = (i < i0 || !found) ? -1 : i - bd;
      }
      lds_barrier();
    }
    if (!SMALL) {
      for (int q = threadIdx.x; q < w1 - w0; q += NT) {
        cum[w0 + q] = ring[(w0 + q) & RM];
        back[w0 + q] = bkw[q];
      }
      lds_barrier();  // the next window restages lsw / bkw
    }
  }
  __syncthreads();  // cum / back global stores (long sequences) visible to the whole workgroup

  // ------------------------------------------------------------ last beat
  NC_BEAT_T(3);
  for (int i = threadIdx.x; i < N; i += NT) {
    const double x = cum[i];
    const bool left = i > 0 ? (x > cum[i - 1]) : false;
    const bool right = i < N - 1 ? (x >= cum[i + 1]) : true;
    marks[i] = (left && right) ? 1 : 0;
  }
  int cnt = 0;
  for (int i = threadIdx.x; i < N; i += NT) cnt += marks[i];
  cnt = block_sum_i<NT>(cnt, bs);
  int tail = N - 1;
  if (cnt > 0) {
    double med;
    if (cnt <= NT) {
      // few peaks (short sequences): compact their scores, then every peak counts the scores
      // below / not above its own; the order statistics cnt/2 (and cnt/2 - 1) are the scores
      // whose [lt, le) rank interval holds them.  One pass, two barriers, in place of the
      // 8-pass radix select (same values: the k-th smallest in f64 order)
      double* cv = dp_best;  // free after the DP
      if (threadIdx.x == 0) sh_int[0] = 0;
      __syncthreads();
      for (int i = threadIdx.x; i < N; i += NT)
        if (marks[i]) cv[atomicAdd(&sh_int[0], 1)] = cum[i];
      __syncthreads();
      const int k1 = (cnt - 1) / 2, k2 = cnt / 2;
      if ((int)threadIdx.x < cnt) {
        const double v = cv[threadIdx.x];
        int lt = 0, le = 0;
        for (int j = 0; j < cnt; ++j) {
          const double u = cv[j];
          lt += u < v;
          le += u <= v;
        }
        if (lt <= k1 && k1 < le) sel_med[0] = v;
        if (lt <= k2 && k2 < le) sel_med[1] = v;
      }
      __syncthreads();
      med = (cnt & 1) ? sel_med[1] : (sel_med[0] + sel_med[1]) / 2.0;
    } else if (cnt & 1) {
      med = block_kth_flagged<NT>(cum, marks, N, cnt / 2, hist, bs);
    } else {
      const double lo = block_kth_flagged<NT>(cum, marks, N, cnt / 2 - 1, hist, bs);
      const double hi = block_kth_flagged<NT>(cum, marks, N, cnt / 2, hist, bs);
      med = (lo + hi) / 2.0;
    }
    const double thr2 = 0.5 * med;
    int t = -1;
    for (int i = threadIdx.x; i < N; i += NT)
      if (marks[i] && cum[i] >= thr2) t = max(t, i);
    t = block_max_i<NT>(t, bs);
    if (t >= 0) tail = t;
  }

  // ------------------------------------------------------------ backtrack
  NC_BEAT_T(4);
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += NT) marks[i] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    int n = tail;
    while (n >= 0) {
      marks[n] = 1;
      n = back[n];
    }
  }
  __syncthreads();

  // ------------------------------------------------------------ ordered beat list (into back[])
  const int chunk = (N + NT - 1) / NT;
  const int c0 = min(N, (int)threadIdx.x * chunk), c1 = min(N, c0 + chunk);
  int mine = 0;
  for (int i = c0; i < c1; ++i) mine += marks[i];
  int nb = 0;
  int pos = block_exclusive_scan<NT>(mine, nb, bs);
  __syncthreads();
  for (int i = c0; i < c1; ++i)
    if (marks[i]) back[pos++] = i;
  __syncthreads();

  // ------------------------------------------------------------ trim (0.5 RMS of smoothed beat scores)
  NC_BEAT_T(5);
  double thr3 = 0.0;
  if (a.trim) {
    double e2 = 0.0;
    const int cntsm = min(N, nb + 2);
    for (int j = threadIdx.x; j < cntsm; j += NT) {
      double v;
      if (j < nb) {
        const double xm = j > 0 ? ls[back[j - 1]] : 0.0;
        const double xp = j + 1 < nb ? ls[back[j + 1]] : 0.0;
        v = (0.5 * xm + ls[back[j]]) + 0.5 * xp;
      } else if (j == nb) {
        v = 0.5 * ls[back[nb - 1]];
      } else {
        v = 0.0;
      }
      e2 += v * v;
    }
    e2 = block_sum<NT>(e2, bs);
    thr3 = 0.5 * sqrt(e2 / (double)cntsm);
  }
  int lo = N, hi = -1;
  for (int i = threadIdx.x; i < N; i += NT)
    if (ls[i] > thr3) {
      lo = min(lo, i);
      hi = max(hi, i);
    }
  lo = block_min_i<NT>(lo, bs);
  hi = block_max_i<NT>(hi, bs);
  // kept beats: lo <= frame <= hi, a contiguous run of the ordered list
  int kfirst = nb, klast = -1;
  for (int j = threadIdx.x; j < nb; j += NT) {
    const int f = back[j];
    if (f >= lo && f <= hi) {
      kfirst = min(kfirst, j);
      klast = max(klast, j);
    }
  }
  kfirst = block_min_i<NT>(kfirst, bs);
  klast = block_max_i<NT>(klast, bs);
  const int nkeep = klast >= kfirst ? klast - kfirst + 1 : 0;
  if (threadIdx.x == 0) a.nbeats_out[s] = nkeep;
  if (a.beats_out)
    for (int j = threadIdx.x; j < nkeep; j += NT) a.beats_out[off + j] = back[kfirst + j];
  NC_BEAT_T(6);
  NC_BEAT_DUMP();
  (void)sh_int;
}

// ---------------------------------------------------------------------------------------------
// nc tempo prior (pipeline.py:174-183): median of the valid source window tempos
// x (src_duration / nc_duration), or 120 when no source window is valid.
template <int NT>
__global__ __launch_bounds__(NT) void nc_prior_kernel(const double* bpm, const int* nbeats,
                                                      const uint8_t* active, const int* src_w0,
                                                      const int* src_w1, const int64_t* src_len,
                                                      const int64_t* nc_len, int sr, int min_beats,
                                                      double* prior_out) {
  __shared__ BlockScratch<NT> bs;
  __shared__ int hist[256];
  __shared__ uint8_t flag[4096];
  const int p = blockIdx.x;
  const int w0 = src_w0[p], w1 = src_w1[p];
  const int n = min(w1 - w0, 4096);
  int cnt = 0;
  for (int i = threadIdx.x; i < n; i += NT) {
    const int w = w0 + i;
    const uint8_t f = (active == nullptr || active[w]) && nbeats[w] >= min_beats;
    flag[i] = f;
    cnt += f;
  }
  cnt = block_sum_i<NT>(cnt, bs);
  const double nc_dur = (double)nc_len[p] / (double)sr;
  const double src_dur = (double)src_len[p] / (double)sr;
  double prior = 120.0;
  if (cnt > 0 && nc_dur > 0 && src_dur > 0) {
    double med;
    if (cnt & 1) {
      med = block_kth_flagged<NT>(bpm + w0, flag, n, cnt / 2, hist, bs);
    } else {
      const double lo = block_kth_flagged<NT>(bpm + w0, flag, n, cnt / 2 - 1, hist, bs);
      const double hi = block_kth_flagged<NT>(bpm + w0, flag, n, cnt / 2, hist, bs);
      med = (lo + hi) / 2.0;
    }
    prior = med * (src_dur / nc_dur);
  }
  if (threadIdx.x == 0) prior_out[p] = prior;
}

// ---------------------------------------------------------------------------------------------
// tempo.py:165-172: t = frames*hop/sr, ibis = diff(t), keep > 0.05 s; counts < min -> 0.
template <int NT>
__global__ __launch_bounds__(NT) void ibi_from_beats_kernel(const int* beats, const int64_t* off,
                                                            const int* nbeats, int sr, int hop,
                                                            int min_ibis, double* ibi_out, int* n_ibi) {
  __shared__ BlockScratch<NT> bs;
  const int s = blockIdx.x;
  const int nb = nbeats[s];
  const int64_t o = off[s];
  if (nb < min_ibis + 1) {
    if (threadIdx.x == 0) n_ibi[s] = 0;
    return;
  }
  const int m = nb - 1;
  const int chunk = (m + NT - 1) / NT;
  const int c0 = min(m, (int)threadIdx.x * chunk), c1 = min(m, c0 + chunk);
  auto ibi = [&](int j) {
    const double t0 = (double)((long long)beats[o + j] * hop) / (double)sr;
    const double t1 = (double)((long long)beats[o + j + 1] * hop) / (double)sr;
    return t1 - t0;
  };
  int mine = 0;
  for (int j = c0; j < c1; ++j) mine += ibi(j) > 0.05;
  int tot = 0;
  int pos = block_exclusive_scan<NT>(mine, tot, bs);
  for (int j = c0; j < c1; ++j) {
    const double v = ibi(j);
    if (v > 0.05) ibi_out[o + pos++] = v;
  }
  if (threadIdx.x == 0) n_ibi[s] = tot < min_ibis ? 0 : tot;
}

// ---------------------------------------------------------------------------------------------
int launch_tempo_beats(Context& ctx, BeatArgs a, int n_seq, int max_len, hipStream_t st) {
  if (n_seq <= 0) return 0;
  a.max_len = max_len;
  a.max_tempo = 320.0;
  a.tightness = 100.0f;
  a.sr = a.sr ? a.sr : ctx.sr;
  // longest possible window table / penalty table: 2P+1 with P <= acw-1
  a.tab_cap = 2 * (a.acw - 1) + 2;
  const size_t tab = al16((size_t)a.tab_cap * sizeof(double));
  const size_t small_lds = tab + (size_t)max_len * (8 + 8 + 4 + 1) + 16;
  if (small_lds <= 64 * 1024) {
    {
      KTimer kt_(ctx, "tempo_beat", st);
      a.span = kt_.span();
      for (int rep = 0; rep < NC_PROBE_REPS(0); ++rep)
        hipLaunchKernelGGL((tempo_beat_kernel<256, true>), dim3(n_seq), dim3(256), small_lds, st, a);
    }
  } else {
    if (!a.ws_ls || !a.ws_cum || !a.ws_back || !a.ws_marks) {
      set_error("tempo_beats: long sequences need the global workspace");
      return -3;
    }
    // LDS ring of cumulative scores: >= dmax + B = 2P + round(P/2) frames, P <= acw - 1
    int ring = 1;
    while (ring < (a.tab_cap / 2) * 5 / 2 + 2) ring <<= 1;
    a.ring_cap = ring;
    const size_t lds = tab + (size_t)ring * sizeof(double) + (size_t)kBeatWin * (sizeof(double) + sizeof(int));
    if (lds > 150 * 1024) {
      set_error("tempo_beats: tempogram window too long");
      return -2;
    }
    {
      KTimer kt_(ctx, "tempo_beat", st);
      a.span = kt_.span();
      a.phase = 1;
      hipLaunchKernelGGL((tempo_beat_kernel<1024, false>), dim3(n_seq), dim3(1024), lds, st, a);
      hipLaunchKernelGGL((beat_localscore_kernel<256>), dim3((unsigned)((max_len + 255) / 256), n_seq), dim3(256),
                         (size_t)a.tab_cap * sizeof(double), st, a);
      a.phase = 2;
      hipLaunchKernelGGL((tempo_beat_kernel<1024, false>), dim3(n_seq), dim3(1024), lds, st, a);
    }
  }
  NC_HIP(hipGetLastError());
  return 0;
}

int launch_nc_prior(const double* bpm, const int* nbeats, const uint8_t* active, const int* src_w0,
                    const int* src_w1, const int64_t* src_len, const int64_t* nc_len, int n_pairs,
                    double* prior_out, hipStream_t st, int sr) {
  if (n_pairs <= 0) return 0;
  hipLaunchKernelGGL((nc_prior_kernel<256>), dim3(n_pairs), dim3(256), 0, st, bpm, nbeats, active, src_w0,
                     src_w1, src_len, nc_len, sr, 4, prior_out);
  NC_HIP(hipGetLastError());
  return 0;
}

int launch_ibi_from_beats(const int* beats, const int64_t* off, const int* nbeats, int n_seq, int hop,
                          int min_ibis, double* ibi_out, int* n_ibi, hipStream_t st, int sr) {
  if (n_seq <= 0) return 0;
  hipLaunchKernelGGL((ibi_from_beats_kernel<256>), dim3(n_seq), dim3(256), 0, st, beats, off, nbeats, sr,
                     hop, min_ibis, ibi_out, n_ibi);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

namespace nc {
int launch_tempo_beats_c(Context& ctx, const float* onset, const int64_t* off, const int* len, int n_seq,
                         int max_len, const double* tg, int acw, const double* start_bpm, const int* prior_idx,
                         const uint8_t* active, int hop, int trim, double* bpm_out, int* lag_out,
                         int* nbeats_out, double* margin_out, int* beats_out, int64_t total_frames, void* ws,
                         size_t ws_bytes, hipStream_t st) {
  BeatArgs a{};
  a.onset = onset;
  a.off = off;
  a.len = len;
  a.tg = tg;
  a.acw = acw;
  a.start_bpm = start_bpm;
  a.prior_idx = prior_idx;
  a.active = active;
  a.sr = ctx.sr;
  a.hop = hop;
  a.trim = trim;
  a.bpm_out = bpm_out;
  a.lag_out = lag_out;
  a.nbeats_out = nbeats_out;
  a.margin_out = margin_out;
  a.beats_out = beats_out;
  if (ws && total_frames > 0 && ws_bytes >= (size_t)total_frames * 21) {
    a.ws_ls = static_cast<double*>(ws);
    a.ws_cum = a.ws_ls + total_frames;
    a.ws_back = reinterpret_cast<int*>(a.ws_cum + total_frames);
    a.ws_marks = reinterpret_cast<uint8_t*>(a.ws_back + total_frames);
  }
  (void)ctx;
  return launch_tempo_beats(ctx, a, n_seq, max_len, st);
}
}  // namespace nc

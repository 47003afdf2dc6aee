// melodia.hip — the frame-parallel front end of MELODIA (Salamon & Gomez 2012, essentia's
// PredominantPitchMelodia as the reference calls it at pitch.py:210-215: frameSize 2048, hopSize
// 128, every other parameter at essentia's default), opt-in and PARITY UNPINNED: essentia is not in
// this image, so nothing here is checked against essentia's own output; the CPU restatement that
// the GPU tests compare with is oracle/melodia_ref.py.  Contour tracking and melody selection are
// sequential and run on the host (nightcore_analyzer/melodia.py).
//
// Per frame t of a file (one 256-thread workgroup per frame, frames walked grid-stride):
//   1. samples [t hop - 1024, t hop + 1024) (zero outside the file: essentia's FrameCutter with
//      startFromZero = false), times the normalised symmetric Hann window (Windowing "hann",
//      normalized: 2 w / sum w), zero-padded to 8192 (zeroPadding 3 frameSize);
//   2. |X[k]|, k = 0..4096: the 8192-point real FFT as a 4096-point complex block FFT of the packed
//      frame (the zero-padded three quarters of the stage-1 inputs are compile-time zeros) plus the
//      real split (Spectrum);
//   3. SpectralPeaks: local maxima k in [1, 4095] (|X[k]| > |X[k-1]|, >= |X[k+1]|), parabolic
//      interpolation, the 100 largest by magnitude (ties: lower bin first);
//   4. PitchSalienceFunction: 600 bins of 10 cents from 55 Hz; every peak within 40 dB of the
//      frame's largest adds magnitude * 0.8^h * cos^2(d pi / 20) to the bins d <= 10 around
//      round(120 log2(f / (h + 1) / 55)), h < 20 harmonics (stopping below 55 Hz);
//   5. PitchSalienceFunctionPeaks: local maxima of the salience in bins [round(120 log2(80 / 55)),
//      599] with salience > 0, the largest kSalPk by salience (ties: lower bin first).
// The salience of a bin is summed in a fixed order (contributing harmonic bins ascending, then
// peak-and-harmonic order), so results are deterministic run to run.
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

constexpr int MD_NT = 256;          // threads per frame
constexpr int MD_N = 4096;          // complex FFT points (8192 real)
constexpr int MD_BINS = 4097;       // |X[k]|, k = 0..4096
constexpr int MD_MAXPK = 100;       // SpectralPeaks maxPeaks
constexpr int MD_NH = 20;           // numberHarmonics
constexpr int MD_SAL = 600;         // salience bins (5 octaves of 10 cents)
constexpr int MD_SEMI = 10;         // bins per semitone
constexpr int MD_BUCKETS = MD_SAL + MD_SEMI;  // harmonic bins 0..609 can reach a salience bin
constexpr int MD_SALPK = 128;       // salience peaks kept per frame (kSalPk in ncgpu.h)
constexpr int MD_ENT = MD_MAXPK * MD_NH;

struct MelodiaArgs {
  const float* sig;
  const int64_t* file_off;
  const int64_t* file_len;
  const int64_t* frame_base;  // [n_files + 1]
  int n_files;
  int64_t total_frames;
  int hop;
  float sr;
  const float* win;           // [2048] normalised Hann
  const float2* tw;           // 8192-entry twiddle table
  int sal_min_bin;            // round(120 log2(minFrequency / 55))
  int* pk_count;              // [total_frames]
  int* pk_bin;                // [total_frames][MD_SALPK]
  float* pk_sal;              // [total_frames][MD_SALPK]
};

// monotone float -> uint (larger float -> larger uint), for sort keys
__device__ __forceinline__ unsigned md_ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// ascending bitonic sort of n (a power of two, <= 4 * 1024) keys in LDS by all MD_NT threads
__device__ void md_bitonic(unsigned long long* key, int n, int tid) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n / 2; i += MD_NT) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long a = key[lo], b = key[hi];
        if ((a > b) == up) {
          key[lo] = b;
          key[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ int md_pow2(int n) {
  int p = 2;
  while (p < n) p <<= 1;
  return p;
}

// 120 log2(f / 55) + 0.5, floored (essentia's frequency-to-cent-bin of PitchSalienceFunction)
// in f64 (round 5): a harmonic whose position lands near a bin boundary is binned as the f64
// oracle bins it (f32 log2f moved some across, the main cause of top-bin disagreements)
__device__ __forceinline__ int md_cent_bin(double f) { return (int)floor(120.0 * log2(f / 55.0) + 0.5); }

__global__ __launch_bounds__(MD_NT) void melodia_salience_kernel(MelodiaArgs a) {
  __shared__ __attribute__((aligned(16))) float2 fft[LdsSize<MD_N>::value];  // 33.8 KB
  __shared__ float mag[MD_BINS + 3];
  __shared__ double pk_f[MD_MAXPK], pk_a[MD_MAXPK];
  __shared__ double sal[MD_SAL];
  __shared__ int bcount[MD_BUCKETS + 1], bstart[MD_BUCKETS + 1];
  __shared__ int ncand, npk;
  const int tid = threadIdx.x;
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(fft);  // after the spectrum: sort keys
  // after the spectral peaks: salience entries (key = peak * 20 + h, f64 weight), bucketed by
  // harmonic bin
  int* ent_key = reinterpret_cast<int*>(fft);
  double* ent_w = reinterpret_cast<double*>(reinterpret_cast<int*>(fft) + MD_ENT);
  int* ent_pos = reinterpret_cast<int*>(fft) + 3 * MD_ENT;  // bucketed order: index into the entries
  static_assert(4 * MD_ENT * sizeof(int) <= LdsSize<MD_N>::value * sizeof(float2), "entries fit the FFT slot");

  for (int64_t g = blockIdx.x; g < a.total_frames; g += gridDim.x) {
    // file of frame g
    int lo = 0, hi = a.n_files - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.frame_base[mid] <= g) lo = mid;
      else hi = mid - 1;
    }
    const int f = lo;
    const int64_t t = g - a.frame_base[f], L = a.file_len[f];
    const float* x = a.sig + a.file_off[f];
    const int64_t s0 = t * a.hop - 1024;
    // 1-2. windowed, zero-padded frame -> 4096-point block FFT of z[n] = x[2n] + i x[2n + 1]
    FftIn<MD_N, MD_NT> in;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r < 4) {
        const int n = tid + MD_NT * r;
        const int64_t i0 = s0 + 2 * n;
        const float x0 = (i0 >= 0 && i0 < L) ? x[i0] : 0.0f;
        const float x1 = (i0 + 1 >= 0 && i0 + 1 < L) ? x[i0 + 1] : 0.0f;
        in[0][r] = make_float2(x0 * a.win[2 * n], x1 * a.win[2 * n + 1]);
      } else {
        in[0][r] = make_float2(0.0f, 0.0f);
      }
    }
    __syncthreads();  // the previous frame's last LDS reads (salience peaks) are done
    block_fft<MD_N, MD_NT>(in, fft, a.tw, tid);
    // real split: X[k] = E + W_8192^k O, E = (Z[k] + conj Z[N - k]) / 2, O = -i (Z[k] - conj Z[N - k]) / 2
    for (int k = tid; k < MD_BINS; k += MD_NT) {
      const float2 za = fft[lpad(k & (MD_N - 1))];
      const float2 zb = cconj(fft[lpad((MD_N - k) & (MD_N - 1))]);
      const float2 E = cscale(cadd(za, zb), 0.5f);
      const float2 O = cmul_mi(cscale(csub(za, zb), 0.5f));
      const float2 X = cadd(E, cmul(a.tw[k], O));
      mag[k] = sqrtf(fmaf(X.x, X.x, X.y * X.y));
    }
    if (tid == 0) ncand = 0;
    __syncthreads();
    // 3. spectral peaks: candidates (local maxima) -> keys (magnitude descending, bin ascending)
    for (int k = 1 + tid; k < MD_BINS - 1; k += MD_NT) {
      const float l = mag[k - 1], c = mag[k], r = mag[k + 1];
      if (c > l && c >= r && c > 0.0f) {
        const double pos = (double)k + 0.5 * ((double)l - r) / ((double)l - 2.0 * c + r);
        const double val = c - 0.25 * ((double)l - r) * (pos - (double)k);
        const int q = atomicAdd(&ncand, 1);
        keys[q] = ((unsigned long long)(~md_ord((float)val)) << 32) | (unsigned)k;
      }
    }
    __syncthreads();
    const int nc = ncand;
    const int ns = md_pow2(nc);
    for (int i = nc + tid; i < ns; i += MD_NT) keys[i] = ~0ull;
    __syncthreads();
    md_bitonic(keys, ns, tid);
    const int np = min(nc, MD_MAXPK);
    if (tid < np) {
      const int k = (int)(unsigned)(keys[tid] & 0xffffffffu);
      const float l = mag[k - 1], c = mag[k], r = mag[k + 1];
      const double pos = (double)k + 0.5 * ((double)l - r) / ((double)l - 2.0 * c + r);
      pk_a[tid] = c - 0.25 * ((double)l - r) * (pos - (double)k);
      pk_f[tid] = pos * (double)a.sr / 8192.0;
    }
    for (int b = tid; b <= MD_BUCKETS; b += MD_NT) bcount[b] = 0;
    __syncthreads();
    // 4. salience entries of the peaks within 40 dB of the largest (MD_NH harmonics each, stopping
    // at the first below 55 Hz), counted per harmonic bin
    const double amin = np > 0 ? pk_a[0] * 0.01 : 0.0;
    if (tid < np && pk_a[tid] > amin) {
      for (int h = 0; h < MD_NH; ++h) {
        const int hb = md_cent_bin(pk_f[tid] / (double)(h + 1));
        if (hb < 0) break;
        if (hb < MD_BUCKETS) atomicAdd(&bcount[hb], 1);
      }
    }
    __syncthreads();
    if (tid == 0) {  // bucket starts (610 buckets: one thread, cheap beside the FFT)
      int s = 0;
      for (int b = 0; b < MD_BUCKETS; ++b) {
        bstart[b] = s;
        s += bcount[b];
        bcount[b] = 0;
      }
      bstart[MD_BUCKETS] = s;
    }
    __syncthreads();
    if (tid < np && pk_a[tid] > amin) {
      for (int h = 0; h < MD_NH; ++h) {
        const int hb = md_cent_bin(pk_f[tid] / (double)(h + 1));
        if (hb < 0) break;
        if (hb < MD_BUCKETS) {
          const int e = bstart[hb] + atomicAdd(&bcount[hb], 1);
          ent_key[e] = tid * MD_NH + h;
          ent_w[e] = pk_a[tid] * pow(0.8, (double)h);
        }
      }
    }
    __syncthreads();
    // within a bucket, entries in (peak, harmonic) order: insertion sort of the few entries
    for (int b = tid; b < MD_BUCKETS; b += MD_NT) {
      const int e0 = bstart[b], e1 = bstart[b + 1];
      for (int i = e0; i < e1; ++i) ent_pos[i] = i;
      for (int i = e0 + 1; i < e1; ++i) {
        const int v = ent_pos[i];
        int j = i - 1;
        while (j >= e0 && ent_key[ent_pos[j]] > ent_key[v]) {
          ent_pos[j + 1] = ent_pos[j];
          --j;
        }
        ent_pos[j + 1] = v;
      }
    }
    __syncthreads();
    // salience of bin b: the entries of harmonic bins b - 10 .. b + 10, ascending
    for (int b = tid; b < MD_SAL; b += MD_NT) {
      double s = 0.0;
      for (int hb = max(0, b - MD_SEMI); hb <= b + MD_SEMI; ++hb) {
        const int d = hb > b ? hb - b : b - hb;
        const double cw = cos((double)d / MD_SEMI * 3.141592653589793 / 2.0);
        const double nbw = cw * cw;
        for (int i = bstart[hb]; i < bstart[hb + 1]; ++i) s += ent_w[ent_pos[i]] * nbw;
      }
      sal[b] = s;
    }
    if (tid == 0) npk = 0;
    __syncthreads();
    // 5. salience peaks in [sal_min_bin, 599]
    for (int b = max(a.sal_min_bin, 0) + tid; b < MD_SAL; b += MD_NT) {
      const double c = sal[b];
      const double l = b > 0 ? sal[b - 1] : -INFINITY;
      const double r = b + 1 < MD_SAL ? sal[b + 1] : -INFINITY;
      if (c > l && c >= r && c > 0.0) {
        const int q = atomicAdd(&npk, 1);
        keys[q] = ((unsigned long long)(~md_ord((float)c)) << 32) | (unsigned)b;
      }
    }
    __syncthreads();
    const int nq = npk;
    const int nqs = md_pow2(nq);
    for (int i = nq + tid; i < nqs; i += MD_NT) keys[i] = ~0ull;
    __syncthreads();
    md_bitonic(keys, nqs, tid);
    const int nout = min(nq, MD_SALPK);
    if (tid < nout) {
      const int b = (int)(unsigned)(keys[tid] & 0xffffffffu);
      a.pk_bin[g * MD_SALPK + tid] = b;
      a.pk_sal[g * MD_SALPK + tid] = (float)sal[b];
    }
    if (tid == 0) a.pk_count[g] = nout;
  }
}

int launch_melodia_salience(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                            const int64_t* frame_base, int n_files, int64_t total_frames, int hop, float sr,
                            const float* win, int sal_min_bin, int* pk_count, int* pk_bin, float* pk_sal,
                            hipStream_t st) {
  if (total_frames <= 0 || n_files <= 0) return 0;
  if (hop <= 0 || sr <= 0.0f || !win) {
    set_error("melodia_salience: hop and sample rate must be positive, win non-null");
    return -2;
  }
  MelodiaArgs a;
  a.sig = sig;
  a.file_off = file_off;
  a.file_len = file_len;
  a.frame_base = frame_base;
  a.n_files = n_files;
  a.total_frames = total_frames;
  a.hop = hop;
  a.sr = sr;
  a.win = win;
  a.tw = ctx.t.tw;
  a.sal_min_bin = sal_min_bin;
  a.pk_count = pk_count;
  a.pk_bin = pk_bin;
  a.pk_sal = pk_sal;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(total_frames, (int64_t)ctx.num_cu * 2));
  {
    KTimer kt_(ctx, "melodia_salience", st);
    hipLaunchKernelGGL(melodia_salience_kernel, dim3(grid), dim3(MD_NT), 0, st, a);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc

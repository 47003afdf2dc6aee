// spectral.hip — per-file spectral statistics behind spectral.analyze
// (spectral.py:52-94): one |STFT| pass (2048 / 512, periodic Hann, centred,
// zero pad) feeding librosa.feature.spectral_centroid, spectral_rolloff(0.85),
// feature.rms, the five |S| band means and the per-bin mean of
// amplitude_to_db(|S|, ref=np.max, top_db=80).  Files are at their native rate
// (the reference loads with sr=None); only the bin spacing and band edges change.
//
// MI355X layout (the librosa path materialises a complex64 1025 x T matrix per
// call and walks it four times; here every frame is transformed once):
//   spectral_frames_kernel  persistent workgroups of SF_WAVES waves, one frame per
//                           wave, contiguous frame ranges (the 4x overlap is served
//                           by the XCD's L2); 1024-point complex wave FFT of the
//                           packed real frame (the stft.hip plan), real split in
//                           registers, |X| into the wave's LDS slot.  Per frame:
//                           the dB row (coalesced 4 KB store), f64 centroid, the
//                           rolloff bin (wave scan of lane-contiguous f32 runs),
//                           the five band sums, max |X| and the frame RMS.
//   spectral_file_kernel    one workgroup per file: frame records -> sums, ref; the
//                           frame-RMS mean / variance / 75th percentile / decay.
//   spectral_bins_kernel    (frame block, file): sum_t max(dB[t][k] - dB(ref), -80)
//                           per bin, a pure HBM stream of the dB rows.
//   spectral_bins_finish    per (file, bin): the block partials in a fixed order.
// Everything is deterministic (no float atomics).
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

// 16 waves (four per SIMD at 110 VGPRs; 147 KB of LDS with full exchange slots): 3.95 -> 3.58 ms
// per 128 3-min files against 14 (round 4, profiles/r4_spectral_waves_ab.txt), outputs unchanged
constexpr int SF_WAVES = 16;
constexpr int SF_THREADS = SF_WAVES * 64;
constexpr int SF_BINS = 1025;
constexpr int SF_ROW = 1028;  // dB row stride (floats): 16-byte aligned rows
constexpr int SF_REC = 8;     // per-frame record: centroid, rolloff Hz, 5 band sums, max |X|
constexpr int SF_NBANDS = 5;
using SfTw = StagedTw<1024>;

struct SpecArgs {
  const float* sig;
  const int64_t* file_off;
  const int64_t* file_len;
  const int64_t* frame_base;  // [n_files + 1]
  const double* bin_hz;       // [n_files]  np.fft.rfftfreq spacing 1 / (2048 * (1 / sr))
  const int* band_bins;       // [n_files][5][2]  [lo, hi) bins of each band mask
  int n_files;
  int64_t total_frames;
  float roll_percent;
  float* rms_out;             // [total_frames]
  float* db_rows;             // [total_frames][SF_ROW]  10 log10(max(1e-10, |X|^2))
  double* rec;                // [total_frames][SF_REC]
  const float2* tw;
  const float* hann2048;
  unsigned long long* span = nullptr;  // nc_profile execution span (nc_device.h)
};

__device__ __forceinline__ int sf_file_of(const int64_t* base, int n, int64_t g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (base[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__host__ __device__ __forceinline__ int sf_al4(int n) { return (n + 3) & ~3; }

static size_t spectral_frames_lds_bytes() {
  return (size_t)sf_al4(SfTw::size) * sizeof(float2) + (size_t)SF_WAVES * LdsSize<1024>::value * sizeof(float2);
}

__global__ __launch_bounds__(SF_THREADS) void spectral_frames_kernel(SpecArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* sh_tw = reinterpret_cast<float2*>(smem);
  const int lane0 = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float2* fftbuf = sh_tw + sf_al4(SfTw::size) + wave * LdsSize<1024>::value;

  __shared__ int sh_next;  // the workgroup's frame queue (WgFrameQueue)
  if (threadIdx.x == 0) sh_next = 0;
  fill_staged_tw<1024>(sh_tw, a.tw, threadIdx.x, SF_THREADS);
  __syncthreads();

  const int64_t n_groups = (a.total_frames + SF_WAVES - 1) / SF_WAVES;
  const int64_t gb = n_groups * blockIdx.x / gridDim.x, ge = n_groups * (blockIdx.x + 1) / gridDim.x;
  // The workgroup's frames [f0, f1) go to its waves one at a time (WgFrameQueue, the stft_mel
  // scheme); a wave's frames rise: the file and its descriptors (bounds, length, offset, band
  // bins) are reloaded only when g crosses into a later file, instead of a binary search and a
  // chain of dependent loads per frame
  const int64_t f0 = gb * SF_WAVES, f1 = std::min<int64_t>(ge * SF_WAVES, a.total_frames);
  WgFrameQueue fq(&sh_next, lane0);
  int f = -1;
  int64_t fb = 0, fe = -1, L = 0, off = 0;
  int blo[SF_NBANDS], bhi[SF_NBANDS];
  for (;;) {
    const int64_t g = f0 + fq.take(lane0);
    if (g >= f1) break;
    if (g >= fe) {
      if (f < 0) {
        f = sf_file_of(a.frame_base, a.n_files, g);
      } else {
        do ++f;
        while (f + 1 < a.n_files && a.frame_base[f + 1] <= g);
      }
      f = uniform32(f);
      fb = uniform64(a.frame_base[f]);
      fe = uniform64(a.frame_base[f + 1]);
      L = uniform64(a.file_len[f]);
      off = uniform64(a.file_off[f]);
      const int* bb = a.band_bins + f * 2 * SF_NBANDS;
#pragma unroll
      for (int b = 0; b < SF_NBANDS; ++b) {
        blo[b] = uniform32(bb[2 * b]);
        bhi[b] = uniform32(bb[2 * b + 1]);
      }
    }
    const int64_t t = g - fb;
    const float* x = a.sig + off;
    const int64_t s0 = t * 512 - 1024;

    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const float* hann = a.hann2048;
    FftIn<1024> in;
    double ss64 = 0.0;  // sum of x^2 over the raw frame (feature.rms, spectral.py:59,76)
    if (s0 >= 0 && s0 + 2048 <= L && ((off & 1) == 0)) {
      const float2* x2 = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = lane + 64 * r;
        const float2 v = x2[n];
        const float2 h = reinterpret_cast<const float2*>(hann)[n];
        ss64 = fma((double)v.x, (double)v.x, ss64);
        ss64 = fma((double)v.y, (double)v.y, ss64);
        in[0][r] = make_float2(v.x * h.x, v.y * h.y);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = lane + 64 * r;
        const int64_t i0 = s0 + 2 * n;
        const float x0 = (i0 >= 0 && i0 < L) ? x[i0] : 0.0f;
        const float x1 = (i0 + 1 >= 0 && i0 + 1 < L) ? x[i0 + 1] : 0.0f;
        ss64 = fma((double)x0, (double)x0, ss64);
        ss64 = fma((double)x1, (double)x1, ss64);
        in[0][r] = make_float2(x0 * hann[2 * n], x1 * hann[2 * n + 1]);
      }
    }
    stockham_stage_regs<1024, 16, 1, 64, false, 0, 0>(in, fftbuf, sh_tw, lane);
    stockham_stage<1024, 16, 16, 64, false, 0, 0>(fftbuf, sh_tw, lane);
    float2 v[4][4];
    fft1024_last_mirror<SfTw::s3>(fftbuf, sh_tw, lane, v);
    float* mag = reinterpret_cast<float*>(fftbuf);  // |X[k]|, k in [0, 1024] (all Z reads precede)
    rsplit_mirror<SfTw::split, true, true>(v, sh_tw, lane, [&](int k, float2 X, float2 XN) {
      mag[k] = sqrtf(fmaf(X.x, X.x, X.y * X.y));
      mag[1024 - k] = sqrtf(fmaf(XN.x, XN.x, XN.y * XN.y));
    });

    // coalesced pass, k = lane + 64 j: dB row, l1 norm, first moment, bands, max
    float* row = a.db_rows + g * SF_ROW;
    double l1 = 0.0, m1 = 0.0;
    float band[SF_NBANDS] = {0.f, 0.f, 0.f, 0.f, 0.f};
    float mx = 0.0f;
    // (classifying each 64-bin step against the uniform band edges on scalar branches measured
    // 9 % slower: 5.19 against 4.78 ms per 128 files)
    auto bin = [&](int k) {
      const float s = mag[k];
      row[k] = db10_floor(s * s);  // = 10 log10f(max(1e-10, s^2)), bit for bit
      l1 += (double)s;
      m1 = fma((double)k, (double)s, m1);
      mx = fmaxf(mx, s);
#pragma unroll
      for (int b = 0; b < SF_NBANDS; ++b) band[b] += (k >= blo[b] && k < bhi[b]) ? s : 0.0f;
    };
#pragma unroll
    for (int j = 0; j < 16; ++j) bin(lane + 64 * j);
    if (lane == 0) bin(1024);
    mx = wave_max_u(mx);

    // rolloff: lane l holds bins [16 l, 16 l + 16) (lane 63 also bin 1024) as an f32 running sum
    float run[17];
    const float4* m4 = reinterpret_cast<const float4*>(mag + 16 * lane);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 u = m4[q];
      run[4 * q] = u.x;
      run[4 * q + 1] = u.y;
      run[4 * q + 2] = u.z;
      run[4 * q + 3] = u.w;
    }
    run[16] = lane == 63 ? mag[1024] : 0.0f;
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 17; ++i) {
      acc += run[i];
      run[i] = acc;
    }
    // (a DPP row_shr / row_bcast scan instead measured -0.7 % and changes the f32 association)
    float incl = acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const float total = __shfl(incl, 63, 64);
    const float excl = incl - acc;
    const float thr = a.roll_percent * total;
    int first = 1 << 30;
#pragma unroll
    for (int i = 16; i >= 0; --i)
      if (excl + run[i] >= thr && (i < 16 || lane == 63)) first = 16 * lane + i;
    first = wave_min_i(first);

    // The eight f64 frame sums (l1, m1, the five bands, sum x^2) reduced together through the
    // slot (all reads of mag precede): lane l writes its partials at red[v][l], lane 8 v + j
    // adds red[v][j + 8 i] over i, three DPP steps finish value v in lanes 8 v .. 8 v + 7.
    // One LDS round trip and ~35 instructions instead of eight DPP wave sums (~30 each):
    // spectral_frames 4.78 -> 4.44 ms per 128 3-min files, outputs bit-identical there (f64 sums
    // of f32 values rarely round).
    // Row stride 72: the reads of 32 lanes cover 64 distinct banks.
    double* red = reinterpret_cast<double*>(fftbuf);
    constexpr int RS = 72;
    static_assert(8 * RS * sizeof(double) <= LdsSize<1024>::value * sizeof(float2), "reduction rows fit the slot");
    {
      const double part[8] = {l1, m1, (double)band[0], (double)band[1], (double)band[2], (double)band[3],
                              (double)band[4], ss64};
#pragma unroll
      for (int v = 0; v < 8; ++v) red[v * RS + lane] = part[v];
    }
    const int rv = lane >> 3, rj = lane & 7;
    double fs = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) fs += red[rv * RS + rj + 8 * i];
    fs = dpp_add_f64<0xB1>(fs);   // quad_perm [1,0,3,2]
    fs = dpp_add_f64<0x4E>(fs);   // quad_perm [2,3,0,1]
    fs = dpp_add_f64<0x141>(fs);  // row_half_mirror: the other quad of the 8 lanes
    const double hz = a.bin_hz[f];
    double* r = a.rec + g * SF_REC;
    auto lane_f64 = [&](int l) {
      const long long b = __double_as_longlong(fs);
      const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)b, l), hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
      return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    };
    const double l1w = lane_f64(0), m1w = lane_f64(8);
    if (lane == 0) {
      // util.normalize(norm=1): columns with an l1 norm below tiny(float32) stay unscaled
      r[0] = hz * (l1w < 1.17549435e-38 ? m1w : m1w / l1w);
      r[1] = hz * (double)first;
      r[7] = (double)mx;
    }
    if (rj == 0 && rv >= 2 && rv < 7) r[rv] = fs;                 // the five band sums
    if (lane == 56) a.rms_out[g] = sqrtf((float)(fs / 2048.0));  // feature.rms of the frame
  }
}

// k-th smallest (0-based) of n non-negative floats: 4 passes of 8-bit radix select on the
// IEEE bits (monotonic for x >= 0); hist = 256 ints of LDS.
template <int NT>
__device__ float sf_kth(const float* x, int n, int k, int* hist, BlockScratch<NT>& s) {
  unsigned prefix = 0, mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += NT) {
      const unsigned key = __float_as_uint(x[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // digit pick: 4 bins per lane + a wave prefix scan
      const int lane = threadIdx.x;
      const int h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
      const int sum = h0 + h1 + h2 + h3;
      int incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      const int excl = incl - sum;
      if (excl <= k && k < incl) {
        int r = k - excl, d = 4 * lane;
        if (r >= h0) {
          r -= h0;
          ++d;
          if (r >= h1) {
            r -= h1;
            ++d;
            if (r >= h2) {
              r -= h2;
              ++d;
            }
          }
        }
        s.i[0] = d;
        s.i[1] = r;
      }
    }
    __syncthreads();
    prefix |= (unsigned)s.i[0] << shift;
    mask |= 255u << shift;
    k = s.i[1];
    __syncthreads();
  }
  return __uint_as_float(prefix);
}

// One workgroup per file.  stats[f][0..7] = {sum centroid, sum rolloff Hz, 5 band |S| sums,
// max |S|} from the frame records; stats[f][8..11] = the frame-RMS statistics of
// spectral.py:60-61,77-78: mean and variance (f32 results, f64 sums), np.percentile(rms, 75)
// (numpy's 'linear' rule: virtual index 0.75 (n - 1), the two order statistics by radix
// select, numpy's f32 lerp) and mean(diff(rms[rms > p75])), which telescopes to
// (last loud - first loud) / (n_loud - 1).
template <int NT>
__global__ __launch_bounds__(NT) void spectral_file_kernel(const int64_t* frame_base, const double* rec,
                                                           const float* rms, double* stats) {
  __shared__ BlockScratch<NT> sc;
  __shared__ int hist[256];
  const int f = blockIdx.x;
  const int64_t t0 = frame_base[f], t1 = frame_base[f + 1];
  const int n = (int)(t1 - t0);
  double s[SF_REC - 1] = {0, 0, 0, 0, 0, 0, 0};
  double mx = 0.0, rs = 0.0;
  for (int64_t g = t0 + threadIdx.x; g < t1; g += NT) {
    const double* r = rec + g * SF_REC;
#pragma unroll
    for (int i = 0; i < SF_REC - 1; ++i) s[i] += r[i];
    mx = fmax(mx, r[7]);
    rs += (double)rms[g];
  }
  double* out = stats + f * 12;
#pragma unroll
  for (int i = 0; i < SF_REC - 1; ++i) {
    const double v = block_sum<NT>(s[i], sc);
    if (threadIdx.x == 0) out[i] = v;
  }
  mx = block_max<NT>(mx, sc);
  if (threadIdx.x == 0) out[7] = mx;

  const float* x = rms + t0;
  const float mean = (float)(block_sum<NT>(rs, sc) / n);
  double vs = 0.0;
  for (int i = threadIdx.x; i < n; i += NT) {
    const float d = x[i] - mean;  // numpy: arr - arrmean in f32, then squared
    vs += (double)(d * d);
  }
  const float var = (float)(block_sum<NT>(vs, sc) / n);
  const double vi = 0.75 * n + 0.25 - 1.0;  // numpy _compute_virtual_index(n, 0.75, 1, 1)
  const int lo = (int)floor(vi);
  const float gamma = (float)(vi - lo);
  const float a = sf_kth<NT>(x, n, lo, hist, sc);
  const float b = lo + 1 < n ? sf_kth<NT>(x, n, lo + 1, hist, sc) : a;
  const float diff = b - a;
  const float p75 = gamma >= 0.5f ? b - diff * (1.0f - gamma) : a + diff * gamma;
  int cnt = 0, first = n, last = -1;
  for (int i = threadIdx.x; i < n; i += NT)
    if (x[i] > p75) {
      ++cnt;
      first = min(first, i);
      last = max(last, i);
    }
  cnt = block_sum_i<NT>(cnt, sc);
  first = block_min_i<NT>(first, sc);
  last = block_max_i<NT>(last, sc);
  if (threadIdx.x == 0) {
    out[8] = (double)mean;
    out[9] = (double)var;
    out[10] = (double)p75;
    out[11] = cnt > 1 ? (double)(float)(((double)x[last] - (double)x[first]) / (cnt - 1)) : 0.0;
  }
}

// (frame block, file): partial[f][blk][k] = sum over the block's frames of max(dB - dB(ref), -80).
// Thread x owns bins 4x .. 4x + 3 (one float4 of the 16-byte aligned row; thread 0 also bin
// 1024) and reads SB_U rows per batch, all loads before the adds, so a wave has 4 KB in flight
// instead of 256 bytes; every bin's f64 sum still runs over the frames in order (bit-identical
// to the one-dword-per-bin form: 1.30 -> 0.79 ms per 128 3-min files, round 3).
constexpr int SB_NT = 256;  // (SF_BINS - 1) / 4 bins as float4s
constexpr int SB_U = 4;  // 8: the same (782 against 788 us), 2: 797 us
static_assert(4 * SB_NT == SF_BINS - 1 && SF_ROW % 4 == 0, "spectral_bins: one float4 per thread plus bin 1024");
__global__ __launch_bounds__(SB_NT) void spectral_bins_kernel(const int64_t* frame_base, const float* db_rows,
                                                              const double* stats, int fb, int nblk,
                                                              double* partial, unsigned long long* span) {
  const Span span_(span);
  const int f = blockIdx.y, blk = blockIdx.x;
  const int64_t t0 = frame_base[f] + (int64_t)blk * fb, t1 = min(frame_base[f + 1], t0 + fb);
  if (t0 >= t1) return;
  // amplitude_to_db -> power_to_db(|S|^2, ref=max|S|^2, amin=1e-10): the f32 reference level
  const float ref = (float)stats[f * 12 + 7];
  const float rdb = 10.0f * log10f(fmaxf(1e-10f, ref * ref));
  const int x = threadIdx.x;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, a4 = 0.0;
  auto add = [&](float4 v) {
    a0 += (double)fmaxf(v.x - rdb, -80.0f);
    a1 += (double)fmaxf(v.y - rdb, -80.0f);
    a2 += (double)fmaxf(v.z - rdb, -80.0f);
    a3 += (double)fmaxf(v.w - rdb, -80.0f);
  };
  int64_t t = t0;
  for (; t + SB_U <= t1; t += SB_U) {
    float4 v[SB_U];
    float e[SB_U];
#pragma unroll
    for (int u = 0; u < SB_U; ++u) {
      const float* row = db_rows + (t + u) * SF_ROW;
      v[u] = reinterpret_cast<const float4*>(row)[x];
      e[u] = row[SF_BINS - 1];  // the same address for every lane: one broadcast load
    }
#pragma unroll
    for (int u = 0; u < SB_U; ++u) {
      add(v[u]);
      a4 += (double)fmaxf(e[u] - rdb, -80.0f);
    }
  }
  for (; t < t1; ++t) {
    const float* row = db_rows + t * SF_ROW;
    add(reinterpret_cast<const float4*>(row)[x]);
    a4 += (double)fmaxf(row[SF_BINS - 1] - rdb, -80.0f);
  }
  double* out = partial + ((size_t)f * nblk + blk) * SF_BINS;
  out[4 * x] = a0;
  out[4 * x + 1] = a1;
  out[4 * x + 2] = a2;
  out[4 * x + 3] = a3;
  if (x == 0) out[SF_BINS - 1] = a4;
}

__global__ void spectral_bins_finish(const int64_t* frame_base, const double* partial, int fb, int nblk,
                                     double* bin_db) {
  const int f = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= SF_BINS) return;
  const int64_t T = frame_base[f + 1] - frame_base[f];
  const int nb = (int)((T + fb - 1) / fb);
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += partial[((size_t)f * nblk + b) * SF_BINS + k];
  bin_db[(size_t)f * SF_BINS + k] = s;
}

// frames per bins-kernel block: at least 32, at most 256 blocks per file
static int spectral_fb(int64_t max_frames) { return (int)std::max<int64_t>(32, (max_frames + 255) / 256); }

size_t spectral_ws_bytes(int64_t total_frames, int n_files, int64_t max_frames) {
  const int fb = spectral_fb(max_frames);
  const int64_t nblk = (max_frames + fb - 1) / fb;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  return al((size_t)total_frames * SF_ROW * sizeof(float)) + al((size_t)total_frames * SF_REC * sizeof(double)) +
         al((size_t)n_files * nblk * SF_BINS * sizeof(double));
}

int launch_spectral(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                    const int64_t* frame_base, const double* bin_hz, const int* band_bins, int n_files,
                    int64_t total_frames, int64_t max_frames, float roll_percent, float* rms_out,
                    double* stats_out, double* bin_db_out, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n_files <= 0 || total_frames <= 0) return 0;
  if (max_frames <= 0 || max_frames > total_frames) {
    set_error("spectral: max_frames must be in [1, total_frames]");
    return -2;
  }
  if (!(roll_percent > 0.0f && roll_percent < 1.0f)) {
    set_error("spectral: roll_percent must lie in (0, 1)");  // spectral_rolloff's own check
    return -2;
  }
  if (ws_bytes < spectral_ws_bytes(total_frames, n_files, max_frames)) {
    set_error("spectral: workspace too small");
    return -2;
  }
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  char* w = static_cast<char*>(ws);
  float* rows = reinterpret_cast<float*>(w);
  w += al((size_t)total_frames * SF_ROW * sizeof(float));
  double* rec = reinterpret_cast<double*>(w);
  w += al((size_t)total_frames * SF_REC * sizeof(double));
  double* partial = reinterpret_cast<double*>(w);

  SpecArgs a{sig, file_off, file_len, frame_base, bin_hz, band_bins, n_files, total_frames, roll_percent,
             rms_out, rows, rec, ctx.t.tw, ctx.t.hann2048};
  const size_t lds = spectral_frames_lds_bytes();
  const int64_t n_groups = (total_frames + SF_WAVES - 1) / SF_WAVES;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(n_groups, (int64_t)ctx.num_cu));
  {
    KTimer kt_(ctx, "spectral_frames", st);
    a.span = kt_.span();
    hipLaunchKernelGGL(spectral_frames_kernel, dim3(grid), dim3(SF_THREADS), lds, st, a);
  }
  NC_HIP(hipGetLastError());
  hipLaunchKernelGGL(spectral_file_kernel<1024>, dim3(n_files), dim3(1024), 0, st, frame_base, rec, rms_out,
                     stats_out);
  NC_HIP(hipGetLastError());
  const int fb = spectral_fb(max_frames);
  const int nblk = (int)((max_frames + fb - 1) / fb);
  {
    KTimer kt_(ctx, "spectral_bins", st);
    hipLaunchKernelGGL(spectral_bins_kernel, dim3(nblk, n_files), dim3(SB_NT), 0, st, frame_base, rows,
                       stats_out, fb, nblk, partial, kt_.span());
  }
  NC_HIP(hipGetLastError());
  hipLaunchKernelGGL(spectral_bins_finish, dim3((SF_BINS + 255) / 256, n_files), dim3(256), 0, st, frame_base,
                     partial, fb, nblk, bin_db_out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc
